"""ctypes binding of the C-ABI (include/viba_hip.h): the HIP LM engine.

:class:`HipEngine` mirrors the part of ``small_thing::Optimizer`` the VI-BA path uses
(lib/small_thing/Optimizer.h): computeGradHess -> ``linearize``, addDamping+factor+solve ->
``damp_factor_solve``, applyStep, computeCost, backup/restore and ``optimize``.
The engine runs entirely on the GPU; there is no CPU fallback: constructing it without the
built library or without a HIP device raises.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from .kinds import NUM_VAR_KINDS, VAR_DATA, VAR_MAX_TANGENT, factor_num_consts, factor_num_vars

P = C.c_void_p
_dp = C.POINTER(C.c_double)


class VbError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"error {code}: {msg}")
        self.code = code


class Settings(C.Structure):
    """Optimizer::Settings, direct-solver subset (lib/small_thing/Optimizer.h:40-91)."""
    _fields_ = [
        ("max_num_iterations", C.c_int32),
        ("stop_if_no_improvement_for", C.c_int32),
        ("distance_from_troubled_iteration", C.c_int32),
        ("max_step_factor_attempts", C.c_int32),
        ("try_sub_step", C.c_int32),
        ("verbose", C.c_int32),
        ("absolute_cost_tolerance", C.c_double),
        ("relative_cost_tolerance", C.c_double),
        ("variables_tolerance", C.c_double),
        ("damping", C.c_double),
        ("damping_adjust_on_fail", C.c_double),
        ("damping_adjust_on_good_step", C.c_double),
        ("damping_adjust_on_average_step", C.c_double),
        ("damping_max", C.c_double),
        ("damping_min", C.c_double),
        ("min_relative_cost_reduction", C.c_double),
        ("step_factor_decrease", C.c_double),
        ("min_step_factor_for_good", C.c_double),
    ]

    @staticmethod
    def default(**kw) -> "Settings":
        s = Settings(50, 3, 3, 2, 1, 0, 1e-8, 1e-10, 1e-5, 1e-5, 2.5, 0.7, 1.5, 1e8, 1e-9, 0.3, 0.3,
                     0.7)
        for k, v in kw.items():
            setattr(s, k, v)
        return s


class Summary(C.Structure):
    """Optimizer::Summary (lib/small_thing/Optimizer.h:93-99)."""
    _fields_ = [("initial_cost", C.c_double), ("final_cost", C.c_double),
                ("num_troubled_seqs", C.c_int32), ("largest_troubled_seq", C.c_int32),
                ("num_iterations", C.c_int32),
                # iterations whose full step failed the reduction / failure-rate test (step rescaling)
                ("num_rescaled", C.c_int32)]


class PhaseTimes(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("linearize_ms", "schur_ms", "factor_ms", "solve_ms",
                                          "step_ms", "cost_ms", "total_ms", "rs_update_ms")]


LOG_CB = C.CFUNCTYPE(None, C.c_char_p, P)
PRESTEP_CB = C.CFUNCTYPE(None, C.c_int, P)


def _arr(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def rs_row_poses(imu_t, imu_gyro, imu_accel, rs_mid, rs_half, rs_calib, gravity, rig_pose, rig_vel, rig_rs, cams,
                 obs_rig, obs_cam, obs_row, lib=None, name="vb_rs_row_poses"):
    """SingleSessionProblem::T_bodyImu_world_atImageRow (viba/problem/VisualFactor.cpp:303-327) of every
    observation (rig obs_rig[i], camera record obs_cam[i] of cams, image row obs_row[i]), with the rolling-
    shutter tables of the rigs built from the IMU-0 stream first (vb_rs_row_poses, include/viba_hip.h; on
    the device).  rs_calib: (n_rs, 32) IMU calibration model per table; rig_rs: table of each rig or -1.
    Returns (n_obs, 7) poses.  `lib` / `name` select another library with the same entry (the oracle)."""
    if lib is None:
        from ._lib import load_hip_lib
        lib = load_hip_lib()
    i64, i32, f64 = (lambda a: _arr(a, np.int64)), (lambda a: _arr(a, np.int32)), (lambda a: _arr(a, np.float64))
    it, ig, ia = i64(imu_t), f64(imu_gyro).reshape(-1, 3), f64(imu_accel).reshape(-1, 3)
    rm, rh, rc, g = i64(rs_mid), i64(rs_half), f64(rs_calib).reshape(-1, 32), f64(gravity).reshape(4)
    rp, rv, rr = f64(rig_pose).reshape(-1, 7), f64(rig_vel).reshape(-1, 3), i32(rig_rs)
    cm, orr, oc, ow = f64(cams).reshape(-1, 24), i32(obs_rig), i32(obs_cam), f64(obs_row)
    out = np.zeros((len(orr), 7))
    f = getattr(lib, name)
    f.restype = C.c_int
    f.argtypes = [C.c_int64, P, P, P, C.c_int32, P, P, P, P, C.c_int64, P, P, P, C.c_int64, P, C.c_int64, P, P, P, P]
    ptr = lambda a: a.ctypes.data_as(P)
    rc_ = f(len(it), ptr(it), ptr(ig), ptr(ia), len(rm), ptr(rm), ptr(rh), ptr(rc), ptr(g), len(rp), ptr(rp), ptr(rv),
            ptr(rr), len(cm), ptr(cm), len(orr), ptr(orr), ptr(oc), ptr(ow), ptr(out))
    if rc_ != 0:
        err = getattr(lib, name.split("_")[0] + "_last_error")
        err.restype = C.c_char_p
        raise VbError(rc_, err().decode())
    return out


class CEngineBase:
    """Shared ctypes plumbing for engines exposing the vb_* function family under a prefix."""

    prefix = "vb_"

    def __init__(self, lib: C.CDLL, handle):
        self.lib = lib
        self.h = handle
        self.nvars = [0] * NUM_VAR_KINDS
        self._keep = []

    # ---------------------------------------------------------------- plumbing
    def _fn(self, name, argtypes, restype=C.c_int):
        f = getattr(self.lib, self.prefix + name)
        f.argtypes = [P] + argtypes
        f.restype = restype
        return f

    def _check(self, rc: int):
        if rc != 0:
            raise VbError(rc, self.last_error())

    def last_error(self) -> str:
        err = getattr(self.lib, self.prefix + "last_error")
        err.restype = C.c_char_p
        return err().decode()

    # ---------------------------------------------------------------- problem
    def set_vars(self, kind: int, data, const=None):
        data = _arr(data, np.float64).reshape(-1, VAR_DATA[kind])
        n = data.shape[0]
        c = None if const is None else _arr(const, np.uint8)
        f = self._fn("set_vars", [C.c_int, C.c_int64, _dp, C.POINTER(C.c_uint8)])
        self._check(f(self.h, kind, n, data.ctypes.data_as(_dp),
                      None if c is None else c.ctypes.data_as(C.POINTER(C.c_uint8))))
        self.nvars[kind] = n

    def add_factors(self, kind: int, var_idx, ivals, consts):
        v = _arr(var_idx, np.int32).reshape(-1, factor_num_vars(kind))
        n = v.shape[0]
        iv = _arr(ivals if ivals is not None else np.full(n, -1), np.int32)
        cs = _arr(consts, np.float64).reshape(n, factor_num_consts(kind))
        f = self._fn("add_factors", [C.c_int, C.c_int64, C.POINTER(C.c_int32),
                                     C.POINTER(C.c_int32), _dp])
        self._check(f(self.h, kind, n, v.ctypes.data_as(C.POINTER(C.c_int32)),
                      iv.ctypes.data_as(C.POINTER(C.c_int32)), cs.ctypes.data_as(_dp)))

    def set_rs_tables(self, offsets, samples, interp, gravity):
        off = _arr(offsets, np.int64)
        s, ip, g = (_arr(x, np.float64) for x in (samples, interp, gravity))
        f = self._fn("set_rs_tables", [C.c_int32, C.POINTER(C.c_int64), _dp, _dp, _dp])
        self._check(f(self.h, len(off) - 1, off.ctypes.data_as(C.POINTER(C.c_int64)),
                      s.ctypes.data_as(_dp), ip.ctypes.data_as(_dp), g.ctypes.data_as(_dp)))

    def set_imu_measurements(self, timestamp_ns, gyro, accel):
        """IMU-0 stream for the device rolling-shutter rebuild (vb_set_imu_measurements)."""
        t = _arr(timestamp_ns, np.int64)
        g, a = _arr(gyro, np.float64).reshape(-1, 3), _arr(accel, np.float64).reshape(-1, 3)
        f = self._fn("set_imu_measurements", [C.c_int64, C.POINTER(C.c_int64), _dp, _dp])
        self._check(f(self.h, len(t), t.ctypes.data_as(C.POINTER(C.c_int64)), g.ctypes.data_as(_dp),
                      a.ctypes.data_as(_dp)))

    def set_imu_stream(self, imu: int, timestamp_ns, gyro, accel):
        """Measurement stream of IMU `imu` (vb_set_imu_stream; imu 0 = the IMU-0 stream above)."""
        t = _arr(timestamp_ns, np.int64)
        g, a = _arr(gyro, np.float64).reshape(-1, 3), _arr(accel, np.float64).reshape(-1, 3)
        f = self._fn("set_imu_stream", [C.c_int, C.c_int64, C.POINTER(C.c_int64), _dp, _dp])
        self._check(f(self.h, int(imu), len(t), t.ctypes.data_as(C.POINTER(C.c_int64)), g.ctypes.data_as(_dp),
                      a.ctypes.data_as(_dp)))

    def set_imu_noise(self, imu: int, accel_var, gyro_var):
        """Sample variances of IMU `imu` (ImuNoiseModelParameters accel/gyroSampleVariance)."""
        a, g = _arr(accel_var, np.float64), _arr(gyro_var, np.float64)
        self._check(self._fn("set_imu_noise", [C.c_int, _dp, _dp])(self.h, int(imu), a.ctypes.data_as(_dp),
                                                                     g.ctypes.data_as(_dp)))

    def set_preint_sources(self, kind: int, imu, t0_us, t1_us):
        """--recompute-preint inputs of the inertial factor rows of `kind` (1..3, vb_add_factors order):
        the IMU and the interval [us] each preintegration integrates (InertialFactors.cpp:19-70)."""
        i, a, b = _arr(imu, np.int32), _arr(t0_us, np.int64), _arr(t1_us, np.int64)
        f = self._fn("set_preint_sources", [C.c_int, C.c_int64, C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                                            C.POINTER(C.c_int64)])
        self._check(f(self.h, int(kind), len(i), i.ctypes.data_as(C.POINTER(C.c_int32)),
                      a.ctypes.data_as(C.POINTER(C.c_int64)), b.ctypes.data_as(C.POINTER(C.c_int64))))

    def update_preintegrations(self):
        """computePreIntegration of every registered inertial row at the current calibration."""
        self._check(self._fn("update_preintegrations", [])(self.h))

    def set_recompute_preint(self, on: bool = True):
        """optimize() recomputes the preintegrations at the start of every iteration (--recompute-preint)."""
        self._check(self._fn("set_recompute_preint", [C.c_int])(self.h, int(bool(on))))

    def get_factor_consts(self, kind: int, row: int) -> np.ndarray:
        from .kinds import factor_num_consts
        out = np.zeros(factor_num_consts(kind))
        self._check(self._fn("get_factor_consts", [C.c_int, C.c_int64, _dp])(self.h, int(kind), int(row),
                                                                             out.ctypes.data_as(_dp)))
        return out

    def set_rs_rigs(self, midpoint_us, half_length_us, imu_calib, gravity_var=0):
        """Per-table rebuild inputs (vb_set_rs_rigs): RollingShutterData's midpoint / half length and
        the IMU calibration variable of updateRollingShutterData (InitCalibration.cpp:316-325)."""
        m, hl = _arr(midpoint_us, np.int64), _arr(half_length_us, np.int64)
        c = _arr(imu_calib, np.int32)
        f = self._fn("set_rs_rigs", [C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                     C.POINTER(C.c_int32), C.c_int32])
        self._check(f(self.h, len(m), m.ctypes.data_as(C.POINTER(C.c_int64)),
                      hl.ctypes.data_as(C.POINTER(C.c_int64)), c.ctypes.data_as(C.POINTER(C.c_int32)),
                      int(gravity_var)))

    def update_rs_tables(self):
        """RollingShutterData::compute of every table from the current variables."""
        self._check(self._fn("update_rs_tables", [])(self.h))

    def get_rs_table(self, t: int):
        """(samples (n, 11), interpolants (n - 1, 9)) of table t."""
        n = C.c_int32()
        f = self._fn("get_rs_table", [C.c_int32, C.POINTER(C.c_int32), _dp, _dp])
        self._check(f(self.h, t, C.byref(n), None, None))
        s = np.zeros((n.value, 11))
        ip = np.zeros((max(0, n.value - 1), 9))
        self._check(f(self.h, t, C.byref(n), s.ctypes.data_as(_dp), ip.ctypes.data_as(_dp)))
        return s, ip

    def refine_points(self):
        """refinePoints (PointRefinement.cpp:160-196): ((start cost, end cost), (failures, iterations,
        points with >= 1 iteration))."""
        c = (C.c_double * 2)()
        st = (C.c_int64 * 3)()
        self._check(self._fn("refine_points", [C.c_double * 2, C.c_int64 * 3])(self.h, c, st))
        return (c[0], c[1]), tuple(st)

    def finalize(self):
        self._check(self._fn("finalize", [])(self.h))

    def reduced_order(self) -> int:
        return self._fn("reduced_order", [], C.c_int64)(self.h)

    def total_order(self) -> int:
        return self._fn("total_order", [], C.c_int64)(self.h)

    # ---------------------------------------------------------------- LM building blocks
    def linearize(self, update_cache=True, dont_retry=False) -> float:
        c = C.c_double()
        self._check(self._fn("linearize", [C.c_int, C.c_int, _dp])(
            self.h, int(update_cache), int(dont_retry), C.byref(c)))
        return c.value

    def damp_factor_solve(self, lam: float) -> float:
        m = C.c_double()
        self._check(self._fn("damp_factor_solve", [C.c_double, _dp])(self.h, lam, C.byref(m)))
        return m.value

    def gradient_dot_step(self, dont_retry=False) -> float:
        b = C.c_double()
        self._check(self._fn("gradient_dot_step", [C.c_int, _dp])(self.h, int(dont_retry),
                                                                   C.byref(b)))
        return b.value

    def solve_with_new_gradient(self):
        self._check(self._fn("solve_with_new_gradient", [])(self.h))

    # ---------------------------------------------------------------- reduced solver
    def set_solver(self, solver_type: int, pcg_max_iterations: int = 40, pcg_desired_residual: float = 1e-10):
        """Optimizer::Settings solverType / pcgMaxIterations / pcgDesiredResidual (Optimizer.h:31-45):
        SOLVER_DIRECT, SOLVER_PCG_TRIVIAL, SOLVER_PCG_JACOBI, SOLVER_PCG_GAUSS_SEIDEL."""
        self._check(self._fn("set_solver", [C.c_int, C.c_int, C.c_double])(
            self.h, int(solver_type), int(pcg_max_iterations), float(pcg_desired_residual)))

    def reduced_layout(self):
        """(kinds, handles, offsets, padded order) of the reduced variables in this handle's ordering
        (vb_reduced_layout)."""
        n, npad = C.c_int64(), C.c_int64()
        f = self._fn("reduced_layout", [P, P, P, C.POINTER(C.c_int64), C.POINTER(C.c_int64)])
        self._check(f(self.h, None, None, None, C.byref(n), C.byref(npad)))
        k = np.zeros(n.value, np.int32)
        hh = np.zeros(n.value, np.int32)
        o = np.zeros(n.value, np.int64)
        self._check(f(self.h, k.ctypes.data, hh.ctypes.data, o.ctypes.data, C.byref(n), C.byref(npad)))
        return k, hh, o, npad.value

    def compute_covariances(self, blocks, damping: float = 1e-5):
        """Optimizer::computeJointCovariances (Optimizer.cpp:503-611): blocks = [[(kind, handle), ...], ...];
        returns ([joint covariance matrix per block], damping used).  vb_compute_covariances /
        ref_compute_covariances; computeCovariances is one variable per block."""
        kinds_, handles = [], []
        start = [0]
        for blk in blocks:
            for k, hh in blk:
                kinds_.append(int(k))
                handles.append(int(hh))
            start.append(len(kinds_))
        k = np.array(kinds_, np.int32)
        hh = np.array(handles, np.int32)
        st = np.array(start, np.int64)
        dims = [[self.var_tangent_dim(int(a), int(b)) for a, b in blk] for blk in blocks]
        sizes = [sum(d) for d in dims]
        out = np.zeros(sum(s * s for s in sizes))
        used = C.c_double()
        f = self._fn("compute_covariances", [C.c_double, C.c_int64, P, P, P, P, C.POINTER(C.c_double)])
        self._check(f(self.h, float(damping), len(blocks), st.ctypes.data, k.ctypes.data, hh.ctypes.data,
                      out.ctypes.data, C.byref(used)))
        covs, o = [], 0
        for s in sizes:
            covs.append(out[o:o + s * s].reshape(s, s, order="F").copy())
            o += s * s
        return covs, used.value

    def var_tangent_dim(self, kind: int, handle: int) -> int:
        """tangent size of one variable (the kind's box-plus dimension; camera records and the IMU
        calibration options decide theirs)"""
        from .kinds import VAR_MAX_TANGENT
        if kind == 4:
            d = self.get_vars(4)[handle]
            return int(d[1]) + int(d[7] != 0) + int(d[8] != 0)
        if kind == 6:
            mask = self.imu_calib_options
            return sum(n for bit, n in ((1, 3), (2, 3), (4, 3), (8, 3), (16, 6), (32, 3), (64, 1), (128, 1)) if mask & bit)
        return VAR_MAX_TANGENT[kind]

    def debug_negate_model_reduction(self, iteration: int):
        """Test fault injection: negate the model cost reduction in LM iteration `iteration` of the next
        optimize (Optimizer.cpp:835-854 branch); -1 disables."""
        self._check(self._fn("debug_negate_model_reduction", [C.c_int])(self.h, int(iteration)))

    def debug_fail_iteration(self, iteration: int):
        """Test fault: iteration `iteration` of the next optimize calls fails as a reduced-system breakdown
        would (VB_E_NUMERIC after the step was applied); the variables must be restored."""
        self._check(self._fn("debug_fail_iteration", [C.c_int])(self.h, int(iteration)))

    def pcg_stats(self):
        """(iterations, relative residual) of the last PCG solve (PCG::Result)."""
        it, rel = C.c_int32(), C.c_double()
        self._check(self._fn("pcg_stats", [C.POINTER(C.c_int32), _dp])(self.h, C.byref(it), C.byref(rel)))
        return it.value, rel.value

    def scale_step(self, f: float):
        self._check(self._fn("scale_step", [C.c_double])(self.h, f))

    def apply_step(self, which=0):
        r = (C.c_double * 3)()
        self._check(self._fn("apply_step", [C.c_int, C.c_double * 3])(self.h, which, r))
        return tuple(r)

    def backup(self):
        self._check(self._fn("backup", [])(self.h))

    def restore(self):
        self._check(self._fn("restore", [])(self.h))

    def get_vars(self, kind: int) -> np.ndarray:
        out = np.zeros((self.nvars[kind], VAR_DATA[kind]))
        self._check(self._fn("get_vars", [C.c_int, _dp])(self.h, kind, out.ctypes.data_as(_dp)))
        return out

    def get_step(self, kind: int, which=0) -> np.ndarray:
        out = np.zeros((self.nvars[kind], VAR_MAX_TANGENT[kind]))
        self._check(self._fn("get_step", [C.c_int, C.c_int, _dp])(
            self.h, which, kind, out.ctypes.data_as(_dp)))
        return out

    # ---------------------------------------------------------------- landmark shards (multi-device)
    def set_landmark_shard(self, lm_begin: int, lm_end: int, is_root: bool):
        self._check(self._fn("set_landmark_shard", [C.c_int64, C.c_int64, C.c_int])(
            self.h, lm_begin, lm_end, int(is_root)))

    def num_params(self) -> int:
        return self._fn("num_params", [], C.c_int64)(self.h)

    def apply_step_raw(self, which=0):
        r = (C.c_double * 3)()
        self._check(self._fn("apply_step_raw", [C.c_int, C.c_double * 3])(self.h, which, r))
        return tuple(r)

    def assemble_reduced(self, lam: float):
        self._check(self._fn("assemble_reduced", [C.c_double])(self.h, lam))

    def factor_solve_reduced(self):
        self._check(self._fn("factor_solve_reduced", [])(self.h))

    def solve_reduced(self):
        self._check(self._fn("solve_reduced", [])(self.h))

    def assemble_new_rhs(self):
        self._check(self._fn("assemble_new_rhs", [])(self.h))

    def back_substitute(self, which=0) -> float:
        m = C.c_double()
        self._check(self._fn("back_substitute_which", [C.c_int, _dp])(self.h, which, C.byref(m)))
        return m.value

    def reduced_buffers(self):
        """(matrix ptr, matrix len, rhs ptr, rhs len) in doubles: device pointers for the HIP
        engine, host pointers for the oracle."""
        m, r = P(), P()
        nm, nr = C.c_int64(), C.c_int64()
        self._check(self._fn("reduced_buffers", [C.POINTER(P), C.POINTER(C.c_int64), C.POINTER(P),
                                                 C.POINTER(C.c_int64)])(
            self.h, C.byref(m), C.byref(nm), C.byref(r), C.byref(nr)))
        return m.value, nm.value, r.value, nr.value

    def shard_tile_range(self):
        a, n = C.c_int64(), C.c_int64()
        self._check(self._fn("shard_tile_range", [C.POINTER(C.c_int64), C.POINTER(C.c_int64)])(
            self.h, C.byref(a), C.byref(n)))
        return a.value, n.value

    def get_gradient(self, kind: int) -> np.ndarray:
        out = np.zeros((self.nvars[kind], VAR_MAX_TANGENT[kind]))
        self._check(self._fn("get_gradient", [C.c_int, _dp])(self.h, kind,
                                                              out.ctypes.data_as(_dp)))
        return out

    # partitioned factorization (vb_set_partition & co.; the oracle restates the protocol)
    def set_partition(self, rank: int, world: int):
        self._check(self._fn("set_partition", [C.c_int, C.c_int])(self.h, rank, world))

    def factor_part(self, which: int):
        self._check(self._fn("factor_part", [C.c_int])(self.h, which))

    def solve_part(self, phase: int):
        self._check(self._fn("solve_part", [C.c_int])(self.h, phase))

    def part_exchange(self, what: int, direction: int):
        """(device pointer, length in doubles) of the engine-owned exchange buffer of `what`
        (0 ROOT tiles, 1 ROOT rows of the forward work vector, 2 ROOT rows of x)."""
        b, n = P(), C.c_int64()
        self._check(self._fn("part_exchange", [C.c_int, C.c_int, C.POINTER(P), C.POINTER(C.c_int64)])(
            self.h, what, direction, C.byref(b), C.byref(n)))
        return b.value, n.value

    def part_info(self):
        out = (C.c_int64 * 5)()
        self._check(self._fn("part_info", [C.c_int64 * 5])(self.h, out))
        return list(out)

    def share_x(self):
        b, n = P(), C.c_int64()
        self._check(self._fn("share_x", [C.POINTER(P), C.POINTER(C.c_int64)])(self.h, C.byref(b), C.byref(n)))
        return b.value, n.value


class HipEngine(CEngineBase):
    """The MI355X LM engine. One instance = one vb_handle = one HIP stream on `device`."""

    prefix = "vb_"

    class Config(C.Structure):
        _fields_ = [("reproj_loss_radius", C.c_double), ("reproj_loss_cutoff", C.c_double),
                    ("imu_loss_radius", C.c_double), ("imu_loss_cutoff", C.c_double),
                    ("imu_calib_options", C.c_int32), ("device", C.c_int32),
                    ("tile", C.c_int32), ("reserved", C.c_int32)]

    def __init__(self, reproj_loss=(1.0, 3.0), imu_loss=(math.inf, math.inf), imu_calib_options=0xFF,
                 device=0, tile=0, precision="fp64"):
        """precision: "fp64" (the reference's arithmetic) or "mixed" (SURVEY config E: fp32 Jacobian
        records and Schur-complement products, fp64 Cholesky; libviba_hip_mixed.so)."""
        from ._lib import load_hip_lib
        if precision not in ("fp64", "mixed"):
            raise ValueError(f"precision must be 'fp64' or 'mixed', not {precision!r}")
        self.precision = precision
        self.imu_calib_options = imu_calib_options
        lib = load_hip_lib(mixed=precision == "mixed")
        cfg = HipEngine.Config()
        lib.vb_default_config.argtypes = [P]
        lib.vb_default_config(C.byref(cfg))
        cfg.reproj_loss_radius, cfg.reproj_loss_cutoff = reproj_loss
        cfg.imu_loss_radius, cfg.imu_loss_cutoff = imu_loss
        cfg.imu_calib_options = imu_calib_options
        cfg.device = device
        cfg.tile = tile
        h = P()
        lib.vb_create.argtypes = [P, C.POINTER(P)]
        lib.vb_create.restype = C.c_int
        super().__init__(lib, None)
        self._check(lib.vb_create(C.byref(cfg), C.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            self.lib.vb_destroy.argtypes = [P]
            self.lib.vb_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def cost(self, comparable=False):
        c = C.c_double()
        st = (C.c_int64 * 3)()
        self._check(self._fn("cost", [C.c_int, _dp, C.c_int64 * 3])(self.h, int(comparable),
                                                                    C.byref(c), st))
        return c.value, tuple(st)

    def optimize(self, settings: Settings | None = None, log=None, prestep=None) -> Summary:
        s = settings or Settings.default()
        out = Summary()
        lcb = LOG_CB(lambda m, u: log(m.decode())) if log else LOG_CB()
        pcb = PRESTEP_CB(lambda i, u: prestep(i)) if prestep else PRESTEP_CB()
        self._check(self._fn("optimize", [C.POINTER(Settings), LOG_CB, PRESTEP_CB, P,
                                          C.POINTER(Summary)])(
            self.h, C.byref(s), lcb, pcb, None, C.byref(out)))
        return out

    def profile_kernel(self, family: int):
        self._check(self._fn("profile_kernel", [C.c_int])(self.h, family))

    def kernel_time(self):
        n, ms = C.c_int64(), C.c_double()
        self._check(self._fn("kernel_time", [C.POINTER(C.c_int64), _dp])(self.h, C.byref(n), C.byref(ms)))
        return n.value, ms.value

    def kernel_busy_time(self):
        """the profiled family's busy time (union of its launches' intervals), ms"""
        ms = C.c_double()
        self._check(self._fn("kernel_busy_time", [_dp])(self.h, C.byref(ms)))
        return ms.value

    def problem_stats(self):
        out = (C.c_int64 * 12)()
        self._check(self._fn("problem_stats", [C.c_int64 * 12])(self.h, out))
        return list(out)

    def factor_schedule_stats(self):
        """[levels, fan-in contributions per factorization, supernodes, two-column supernodes]"""
        out = (C.c_int64 * 4)()
        self._check(self._fn("factor_schedule_stats", [C.c_int64 * 4])(self.h, out))
        return list(out)

    # sparse shard exchange (HIP engine only; the oracle keeps the band of shard_tile_range)
    def shard_tiles(self) -> np.ndarray:
        n = C.c_int64()
        self._check(self._fn("shard_tiles", [C.c_void_p, C.POINTER(C.c_int64)])(self.h, None, C.byref(n)))
        out = np.zeros(n.value, dtype=np.int32)
        if n.value:
            self._check(self._fn("shard_tiles", [C.c_void_p, C.POINTER(C.c_int64)])(
                self.h, out.ctypes.data_as(C.c_void_p), C.byref(n)))
        return out

    def pack_shard_tiles(self):
        """(device pointer, length in doubles) of this shard's tiles packed in shard_tiles order."""
        b, n = P(), C.c_int64()
        self._check(self._fn("pack_shard_tiles", [C.POINTER(P), C.POINTER(C.c_int64)])(
            self.h, C.byref(b), C.byref(n)))
        return b.value, n.value

    def add_tiles(self, tiles_dev: int, n: int, buf_dev: int):
        self._check(self._fn("add_tiles", [C.c_void_p, C.c_int64, C.c_void_p])(self.h, tiles_dev, n, buf_dev))

    # deferred mode: one scalar read per LM iteration in the multi-process controllers (viba_hip.h)
    def set_deferred(self, on: bool):
        self._check(self._fn("set_deferred", [C.c_int])(self.h, int(on)))

    def scalar_slots(self):
        """(device pointer of red[0..24), device pointer of err[0..2)): the phase functions' partial
        scalars in deferred mode (vb_scalar_slots)."""
        r, e = P(), P()
        self._check(self._fn("scalar_slots", [C.POINTER(P), C.POINTER(P)])(self.h, C.byref(r), C.byref(e)))
        return r.value, e.value

    def small_factor_count(self) -> int:
        n = C.c_int64()
        self._check(self._fn("small_factor_count", [C.POINTER(C.c_int64)])(self.h, C.byref(n)))
        return n.value

    def mark_scalars(self):
        self._check(self._fn("mark_scalars", [])(self.h))

    def read_scalars(self, n: int = 17, check: bool = True):
        """red[0, n) on the host, after vb_mark_scalars' point.  check: raise the error the error words
        hold; else return (code, values) so a multi-process caller can agree on it first."""
        out = np.zeros(n)
        rc = self._fn("read_scalars", [_dp, C.c_int])(self.h, out.ctypes.data_as(_dp), n)
        if check:
            self._check(rc)
            return out
        return rc, out

    def error_words(self):
        """the two error bit words behind the last check (vb_error_words)"""
        w = np.zeros(2, np.int32)
        self._check(self._fn("error_words", [C.POINTER(C.c_int32)])(self.h, w.ctypes.data_as(C.POINTER(C.c_int32))))
        return w

    def error_from_words(self, words) -> int:
        """the code two (rank-ORed) error words encode; sets last_error() to its message (vb_error_from_words)"""
        w = np.ascontiguousarray(words, dtype=np.int32)
        return int(self._fn("error_from_words", [C.POINTER(C.c_int32)])(self.h, w.ctypes.data_as(C.POINTER(C.c_int32))))


    def spec_prepare(self) -> bool:
        ok = C.c_int()
        self._check(self._fn("spec_prepare", [C.POINTER(C.c_int)])(self.h, C.byref(ok)))
        return bool(ok.value)

    def spec_linearize(self, dont_retry=False):
        self._check(self._fn("spec_linearize", [C.c_int])(self.h, int(dont_retry)))

    def spec_commit(self, use: bool):
        self._check(self._fn("spec_commit", [C.c_int])(self.h, int(use)))

    def spec_phase_ms(self):
        """(rolling-shutter rebuild ms, linearization ms) of the speculative linearization last committed
        (vb_spec_phase_ms)"""
        out = np.zeros(2)
        self._check(self._fn("spec_phase_ms", [_dp])(self.h, out.ctypes.data_as(_dp)))
        return float(out[0]), float(out[1])

    # partitioned factorization (HIP engine only; include/viba_hip.h vb_set_partition)
    def bench_kernel(self, which: int, iters: int = 200) -> float:
        us = C.c_double()
        self._check(self._fn("bench_kernel", [C.c_int, C.c_int, _dp])(self.h, which, iters, C.byref(us)))
        return us.value

    def stream_ptr(self) -> int:
        """The handle's hipStream_t (vb_stream), for torch.cuda.ExternalStream / RCCL interop."""
        self.lib.vb_stream.restype = P
        self.lib.vb_stream.argtypes = [P]
        return self.lib.vb_stream(self.h)

    def synchronize(self):
        from ._lib import hip_stream_sync
        hip_stream_sync(self.stream_ptr())

    def phase_times(self) -> PhaseTimes:
        t = PhaseTimes()
        self._check(self._fn("last_phase_times", [C.POINTER(PhaseTimes)])(self.h, C.byref(t)))
        return t
