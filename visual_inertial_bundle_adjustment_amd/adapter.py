"""SingleSessionAdapter (viba/single_session/): session data -> the LM problem the engine optimizes.

``SessionAdapter(sd, matcher, settings).build()`` restates ark_vi_ba's problem construction,
``SingleSessionAdapter::initAllVariablesAndFactors`` (SingleSessionAdapter.cpp:67-128) in its default
path (initAllParams, no ground-truth trajectory):

  initRigs                        rigs from the open-loop trajectory              InitRigs.cpp:133-139
  initCamIntrinsics / Extrinsics  per-camera variables over 5 s windows of rigs   InitCalibration.cpp:162-387
  initImuCalibs / ImuExtrinsics   per-IMU variables over the same windows         InitCalibration.cpp:422-579
  initRollingShutterData          per-rig rolling-shutter intervals               InitCalibration.cpp:299-314
  initPointsFromObservations      RANSAC + refinement triangulation (libviba_host) InitPointTracks.cpp:29-63
  addVisualFactors                one factor per inlier observation               VisualFactors.cpp:16-62
  regenerateAllPreintegrations... computePreIntegration per rig pair and IMU      InertialFactors.cpp:19-70
  addInertialFactors              consecutive rigs <= 10 s apart                  InertialFactors.cpp:72-100
  addAllRandomWalkFactors         between consecutive windows of each sensor      RandomWalkFactors.cpp:20-154
  addOmegaPriors                  with > 1 IMU                                    OmegaPriors.cpp:19-31
  add*FactoryCalibPriors          every calibration variable                      FactoryCalibPriors.cpp:22-147

The result is a problem in the engine's row layouts (the fields of synth.GeneratedProblem) plus the
--recompute-preint sources of its inertial rows.  The preintegrations themselves are computed by the
engine on the device (vb_update_preintegrations, preint.hip) right after vb_finalize, from the same IMU
streams and at the same calibration as generatePreintegration; ``load_into`` does that.

Deviation (documented in DESIGN.md): the triangulation uses each observation's rig pose at the frame
timestamp, not the rolling-shutter pose at its image row (Triangulation.h:43 kModelRollingShutter),
because the rolling-shutter tables only exist on the device.  It only changes the initial points.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field

import numpy as np

from . import kinds
from ._lib import load_host_lib
from .session import (CameraCalibration, Matcher, SessionData, imu_scale_mats, se3_inv, se3_mul)
from .synth import GeneratedProblem

# Constants.h / InitCalibration.cpp / InertialFactors.cpp / FactoryCalibPriors.cpp
K_DEFAULT_GRAVITY = 9.81
K_MULTI_IMU_OMEGA_PRIOR_STD = 10.0 * math.pi / 180
K_GROUP_TIME_LENGTH_SEC = 5.0           # kCameraModel / kExtrinsics / kImuCalib GroupTimeLengthSec
K_TIMESTAMP_SLACK_SEC = 1e-3            # initCamIntrinsics
K_RS_TIMESTAMP_SLACK_MS = 2             # initRollingShutterData
K_MAX_INERTIAL_GAP_US = 10_000_000      # kMaxTimeDistanceInertialFactorUs
K_SMALL_INTERVAL_FOR_OMEGA_US = 5_000   # kSmallIntervalForOmegaUs
K_CAM_EXTR_POS_TURNON_STD = 4e-4
K_CAM_EXTR_ROT_TURNON_STD = 0.2 * (math.pi / 180)
# camera_model/RandomWalkCov.cpp, extrinsics_model/RandomWalkCov.cpp
K_CAM_PROJ_RW_VAR = 1e-6
K_CAM_DIST_RW_VAR = 1e-10
K_READOUT_RW_VAR = 1e-10
K_CAM_EXTR_RW_ROT_VAR = 1e-11
K_CAM_EXTR_RW_POS_VAR = (1e-3 * math.pi / 180) ** 2
K_CAM_PROJ_TURNON_STD, K_CAM_DIST_TURNON_STD, K_CAM_RO_TURNON_STD, K_CAM_OFF_TURNON_STD = 1.0, 1e-3, 0.01, 0.01


@dataclass
class InitSettings:
    """The InitSettings fields the adapter reads (viba/common/Settings.h:24-75), reference defaults."""
    rig_start: int = -1
    rig_end: int = -1
    tracking_obs_loss: tuple = (1.0, 3.0)            # kReprojectionErrorHuberLoss{Width,Cutoff}
    imu_loss: tuple = (math.inf, math.inf)           # kImuErrorHuberLossWidth
    estimate_readout_time: bool = False
    estimate_time_offset: bool = False
    cam_intr_constant: bool = False
    cam_extr_constant: bool = False
    imu_calib_constant: bool = False
    imu_extr_constant: bool = False
    imu_calib_options: int = 0xFF                    # ImuCalibrationOptions (all estimated)
    imu_rw_inflate: float = 1.0
    cam_intr_rw_inflate: float = 1.0
    imu_extr_rw_inflate: float = 1.0
    cam_extr_rw_inflate: float = 1.0
    imu_factory_calib_inflate: float = 100.0
    cam_intr_factory_calib_inflate: float = 100.0
    imu_extr_factory_calib_inflate: float = 100.0
    cam_extr_factory_calib_inflate: float = 100.0
    recompute_preint: bool = False


class ImuJacIndices:
    """ImuCalibrationJacobianIndices::computeIndices (imu_types/ImuCalibrationJacobianIndices.h): the
    error-state offsets of the estimated blocks, in the order of the option bits."""

    def __init__(self, mask: int):
        i = 0
        sizes = (("gB", 1, 3), ("aB", 2, 3), ("gS", 4, 3), ("aS", 8, 3), ("gN", 16, 6), ("aN", 32, 3),
                 ("rT", 64, 1), ("gaT", 128, 1))
        for name, bit, n in sizes:
            if mask & bit:
                setattr(self, name, i)
                i += n
            else:
                setattr(self, name, -1)
        self.size = i


@dataclass
class _SensorVar:
    """One calibration variable (SingleSessionProblem's *_addNew bookkeeping)."""
    sensor: int
    window: int
    avg_ts_us: int
    prev: int


@dataclass
class SessionProblem(GeneratedProblem):
    """GeneratedProblem + what the session path adds: rig timestamps, the preintegration sources of the
    inertial rows, the IMU streams, per-sensor calibration variables."""
    rig_ts_us: np.ndarray | None = None
    rig_pose_index: np.ndarray | None = None
    preint_src: dict = field(default_factory=dict)    # kind -> (imu, t0_us, t1_us)
    imu_streams: list = field(default_factory=list)   # ImuSamples per IMU
    imu_noise: list = field(default_factory=list)     # (accel_var3, gyro_var3) per IMU
    windows: list = field(default_factory=list)       # window boundaries (rig indices)
    n_cam: int = 0
    n_imu: int = 0
    triangulated: int = 0
    tried_tracks: int = 0
    point_ids: np.ndarray | None = None               # session point id of each point variable
    reproj_loss: tuple = (1.0, 3.0)
    imu_loss: tuple = (math.inf, math.inf)

    # variable handles of rig i's sensor s (the rigCamToModelIndex_ style maps)
    def cam_var(self, rig: int, s: int) -> int:
        return s * self._n_win + self._rig_win[rig]

    def imu_var(self, rig: int, s: int) -> int:
        return s * self._n_win + self._rig_win[rig]

    def imu_extr_var(self, rig: int, s: int) -> int:
        return (s - 1) * self._n_win + self._rig_win[rig]


def rig_windows(ts_us: np.ndarray, max_len_sec: float) -> list:
    """rigWindowsOfTimeLengthAtMost (InitCalibration.cpp:169-183) over the problem's rigs 0..n-1."""
    max_us = int(max_len_sec * 1e6)
    out, start = [], int(ts_us[0]) - max_us
    for r, t in enumerate(ts_us):
        if int(t) - start >= max_us:
            start = int(t)
            out.append(r)
    out.append(len(ts_us))
    return out


def average_timestamp(ts_us, a, b) -> int:
    """averageTimestampOfRigsInRange (SingleSessionProblem.cpp:540-553)."""
    if b <= a:
        return -1
    s = 0.0
    for t in ts_us[a:b]:
        s += int(t) * 1e-6
    return int((s / (b - a)) * 1e6)


def compensated_gyro_at_end(stream, model, t0_us: int, t1_us: int) -> np.ndarray:
    """PreIntegration::omegaAtEnd (PreIntegration.cpp:272): the compensated gyro of the last step of
    enumIntegrationSteps over [t0, t1] (PreIntegration.cpp:28-111), compensation as
    ImuMeasurementModelParameters::getCompensatedImuMeasurement (.h:87-100)."""
    t = stream.timestamp_ns
    dtG, dtA = int(model[31] * 1e9), int(model[30] * 1e9)
    margin = 1000

    def gt(x):  # measIndex_GT: first sample strictly after x
        i = int(np.searchsorted(t, x, side="right"))
        if i >= len(t):
            raise ValueError("measIndex_GT: unexpected, it == meas.end()")
        return i
    gS, gE = gt(t0_us * 1000 + dtG + margin), gt(t1_us * 1000 + dtG - margin)
    aS, aE = gt(t0_us * 1000 + dtA + margin), gt(t1_us * 1000 + dtA - margin)
    if gS <= 0 or aS <= 0:
        raise ValueError("enumIntegrationSteps: not enough margin at beginning of interval")
    # the loop ends at the step consuming adjA[aE] (then gyro index = first gi with adjG >= adjA[aE])
    # or at the one consuming adjG[gE], whichever comes first
    adjA_end = int(t[aE]) - dtA
    gstar = gS + int(np.searchsorted(t[gS:] - dtG, adjA_end, side="left"))
    gi = min(gstar, gE)
    G, _ = imu_scale_mats(model)
    return np.linalg.solve(G, stream.gyro[gi]) - np.asarray(model[6:9])


class SessionAdapter:
    def __init__(self, sd: SessionData, matcher: Matcher, settings: InitSettings | None = None, row_poses=None):
        self.sd, self.m, self.s = sd, matcher, settings or InitSettings()
        # T_bodyImu_world_atImageRow provider for the triangulation: the device (engine.rs_row_poses,
        # vb_rs_row_poses) unless a caller passes another implementation with the same arguments
        self.row_poses = row_poses
        self.n_cam = len(sd.slam_camera_serials)
        self.n_imu = len(sd.slam_imu_labels)

    # ------------------------------------------------------------------ variables
    def build(self) -> SessionProblem:
        sd, m, s = self.sd, self.m, self.s
        n_rec = len(m.rig_to_pose_index)
        r0 = s.rig_start if s.rig_start >= 0 else 0
        r1 = s.rig_end if s.rig_end >= 0 else n_rec
        if r1 - r0 < 5:  # kMinNumberRigs (SingleSessionAdapter.cpp:132-142)
            raise ValueError(f"Too small problem size, requested rig range {r0}..{r1}")
        nr = r1 - r0
        p = SessionProblem(imu_calib_options=s.imu_calib_options)
        p.n_cam, p.n_imu = self.n_cam, self.n_imu
        p.reproj_loss, p.imu_loss = tuple(s.tracking_obs_loss), tuple(s.imu_loss)
        pose_idx = m.rig_to_pose_index[r0:r1]
        calib_idx = m.rig_to_calib_index[r0:r1]
        ps = sd.inertial_poses
        p.rig_pose_index = pose_idx
        p.rig_ts_us = ps.timestamp_us[pose_idx].astype(np.int64)
        p.vars = [None] * kinds.NUM_VAR_KINDS
        p.const = [None] * kinds.NUM_VAR_KINDS
        # initRigs: T_bodyImu_world = T_w_IMU^-1, vel_world, omega
        p.vars[1] = np.array([se3_inv(ps.T_w_imu[i]) for i in pose_idx]).reshape(nr, 7)
        p.vars[2] = ps.v_w[pose_idx].copy()
        p.vars[3] = ps.omega_bodyimu[pose_idx].copy()
        for k in (1, 2, 3):
            p.const[k] = np.zeros(nr, np.uint8)
        p.vars[8] = np.array([[0.0, 0.0, -K_DEFAULT_GRAVITY, K_DEFAULT_GRAVITY]])
        p.const[8] = np.ones(1, np.uint8)

        win = rig_windows(p.rig_ts_us, K_GROUP_TIME_LENGTH_SEC)
        nw = len(win) - 1
        p.windows = win
        rig_win = np.zeros(nr, np.int64)
        for w in range(nw):
            rig_win[win[w]:win[w + 1]] = w
        p._n_win, p._rig_win = nw, rig_win
        avg = [average_timestamp(p.rig_ts_us, win[w], win[w + 1]) for w in range(nw)]
        last_calib = [calib_idx[win[w + 1] - 1] for w in range(nw)]   # last_in_range: the window's last rig

        # initCamIntrinsics (+ the rigs' rolling-shutter spans)
        cams, self.cam_vars, span = [], [], np.zeros(nr)
        for c in range(self.n_cam):
            ol = m.slam_cam_to_online[c]
            for w in range(nw):
                oc: CameraCalibration = sd.online_calibs[last_calib[w]].cameras[ol]
                is_rs = s.estimate_readout_time or oc.readout_sec is not None
                off = oc.time_offset_sec
                est_ro, est_off = s.estimate_readout_time and is_rs, s.estimate_time_offset and is_rs
                cam_span = ((oc.readout_sec or 0.0) + K_TIMESTAMP_SLACK_SEC if is_rs else 0.0) + \
                    (2.0 * (abs(off) + K_TIMESTAMP_SLACK_SEC) if (est_off or off != 0.0) else 0.0)
                if not cam_span < 1.0:
                    raise ValueError(f"camera {c}: time span {cam_span} >= 1 s")
                cams.append(oc.camera_data(est_ro, est_off))
                self.cam_vars.append(_SensorVar(c, w, avg[w], len(cams) - 2 if w > 0 else -1))
                if cam_span > 0:
                    span[win[w]:win[w + 1]] = np.maximum(span[win[w]:win[w + 1]], cam_span)
        p.vars[4] = np.array(cams).reshape(-1, 24)
        p.const[4] = np.full(len(cams), int(s.cam_intr_constant), np.uint8)
        # initCamExtrinsics
        extr = [sd.online_calibs[last_calib[w]].T_cam_bodyimu[m.slam_cam_to_online[c]]
                for c in range(self.n_cam) for w in range(nw)]
        p.vars[5] = np.array(extr).reshape(-1, 7)
        p.const[5] = np.full(len(extr), int(s.cam_extr_constant), np.uint8)
        # initImuCalibs / initImuExtrinsics (IMU 0 has trivial extrinsics)
        imus = [sd.online_calibs[last_calib[w]].imu_models[m.slam_imu_to_online[i]]
                for i in range(self.n_imu) for w in range(nw)]
        p.vars[6] = np.array(imus).reshape(-1, 32)
        p.const[6] = np.full(len(imus), int(s.imu_calib_constant), np.uint8)
        iext = [sd.online_calibs[last_calib[w]].T_imu_bodyimu[m.slam_imu_to_online[i]]
                for i in range(1, self.n_imu) for w in range(nw)]
        p.vars[7] = np.array(iext).reshape(-1, 7)
        p.const[7] = np.full(len(iext), int(s.imu_extr_constant), np.uint8)
        self.avg, self.nw = avg, nw

        # initRollingShutterData: every rig with a positive span; rig r's table is the r-th of those
        self.rs_table = np.full(nr, -1, np.int64)
        rs_rigs = np.flatnonzero(span > 0)
        self.rs_table[rs_rigs] = np.arange(len(rs_rigs))
        if len(rs_rigs):
            p.rs_mid = np.array([sd.online_calibs[calib_idx[r]].timestamp_us for r in rs_rigs], np.int64)
            p.rs_half = np.array([int(K_RS_TIMESTAMP_SLACK_MS * 1e3 + span[r] * 0.5e6) for r in rs_rigs], np.int64)
            p.rs_calib = np.array([p.imu_var(r, 0) for r in rs_rigs], np.int32)
            imu0 = sd.imu[0]
            p.imu_t, p.imu_gyro, p.imu_accel = imu0.timestamp_ns, imu0.gyro, imu0.accel
        p.imu_streams = list(sd.imu)
        for i in range(self.n_imu):
            nm = sd.imu_noise_models[m.slam_imu_to_factory[i]]
            p.imu_noise.append((np.asarray(nm.accel_sample_var), np.asarray(nm.gyro_sample_var)))

        self._points_and_visual(p, r0, r1)
        self._inertial(p)
        self._random_walks(p)
        self._factory_priors(p)
        for k in range(kinds.NUM_VAR_KINDS):
            if p.vars[k] is None:
                p.vars[k] = np.zeros((0, kinds.VAR_DATA[k]))
                p.const[k] = np.zeros(0, np.uint8)
        p.gt = [v.copy() for v in p.vars]
        return p

    # ------------------------------------------------------------------ points + visual factors
    def _points_and_visual(self, p: SessionProblem, r0: int, r1: int):
        sd, m = self.sd, self.m
        obs = sd.observations
        tracks, seeds, pids = [], [], []
        for pid, pi in m.point_id_to_index.items():   # initPointsFromObservations (filterPointObservations)
            idx = [i for i in m.point_obs[pi] if r0 <= m.obs_to_rig[i] < r1]
            if len(idx) < 3:  # triangulation::kMinInlierObs
                continue
            tracks.append(idx)
            pids.append(pid)
            seeds.append(np.int32(np.int64(pid + 1729).astype(np.int32)))
        p.tried_tracks = len(tracks)
        flat = np.array([i for t in tracks for i in t], np.int64)
        start = np.zeros(len(tracks) + 1, np.int64)
        start[1:] = np.cumsum([len(t) for t in tracks])
        rig = m.obs_to_rig[flat] - r0 if len(flat) else np.zeros(0, np.int64)
        cam = obs.camera_index[flat].astype(np.int64) if len(flat) else np.zeros(0, np.int64)
        camvar = np.array([p.cam_var(int(r), int(c)) for r, c in zip(rig, cam)], np.int32)
        uv = np.ascontiguousarray(obs.uv[flat]).reshape(-1, 2)
        # kModelRollingShutter (Triangulation.h:43): rays and refinements use the rig pose at the
        # observation's image row, T_bodyImu_world_atImageRow (Triangulation.cpp:122-123,184-185), from
        # the rolling-shutter tables updateRollingShutterData builds first (SingleSessionAdapter.cpp:59,64)
        self.row_pose_inputs = (rig, camvar, uv[:, 1].copy())
        Tbw_row = self._row_poses(p, rig, camvar, uv[:, 1])
        Tcw = np.array([se3_mul(p.vars[5][cv], Tbw_row[i]) for i, cv in enumerate(camvar)]).reshape(-1, 7)
        sh = np.ascontiguousarray(obs.sqrt_h[flat]).reshape(-1, 4)
        cams = np.ascontiguousarray(p.vars[4])
        pts = np.zeros((len(tracks), 3))
        ok = np.zeros(len(tracks), np.uint8)
        inl = np.zeros(len(flat), np.uint8)
        seeds = np.array(seeds, np.int32)
        lib = load_host_lib()
        ptr = lambda a: a.ctypes.data_as(C.c_void_p)
        Tcw = np.ascontiguousarray(Tcw)
        lib.vbh_triangulate(len(tracks), ptr(start), ptr(seeds), ptr(Tcw), ptr(camvar), ptr(cams),
                            ptr(uv), ptr(sh), ptr(pts), ptr(ok), ptr(inl))
        # kept for the parity tests (tests/test_session.py against the oracle's triangulatePoint)
        self.triangulation = {"inputs": (start, seeds, Tcw, camvar, cams, uv, sh), "points": pts, "ok": ok,
                              "inliers": inl}
        keep = np.flatnonzero(ok)
        p.triangulated = len(keep)
        p.point_ids = np.array(pids, np.int64)[keep]
        p.vars[0] = pts[keep].reshape(-1, 3)
        p.const[0] = np.zeros(len(keep), np.uint8)
        # addVisualFactors: every inlier observation of every point track
        fv, fi, fc = [], [], []
        for newp, t in enumerate(keep):
            for j in range(start[t], start[t + 1]):
                if not inl[j]:
                    continue
                r, c, cv = int(rig[j]), int(cam[j]), int(camvar[j])
                cd = p.vars[4][cv]
                rs = cd[7] != 0 or cd[6] != 0.0 or cd[8] != 0 or cd[4] != 0  # hasTimeOffset || isRollingShutter
                fv.append((newp, r, cv, cv, r if rs else -1))
                fi.append(int(self.rs_table[r]) if rs else -1)
                fc.append((uv[j, 0], uv[j, 1], *sh[j]))
        self.visual = (np.array(fv, np.int32).reshape(-1, 5), np.array(fi, np.int32), np.array(fc).reshape(-1, 6))

    def _row_pose_args(self, p: SessionProblem, rig, camvar, row) -> tuple:
        """arguments of engine.rs_row_poses: the IMU-0 stream, the rigs' rolling-shutter intervals with
        their IMU calibration models and gravity, the rigs, the cameras, the observations"""
        has_rs = p.rs_mid is not None and len(p.rs_mid) > 0
        e64, e3 = np.zeros(0, np.int64), np.zeros((0, 3))
        return (p.imu_t if has_rs else e64, p.imu_gyro if has_rs else e3, p.imu_accel if has_rs else e3,
                p.rs_mid if has_rs else e64, p.rs_half if has_rs else e64,
                p.vars[6][p.rs_calib] if has_rs else np.zeros((0, 32)), p.vars[8][0], p.vars[1], p.vars[2],
                self.rs_table, p.vars[4], rig, camvar, row)

    def _row_poses(self, p: SessionProblem, rig, camvar, row) -> np.ndarray:
        fn = self.row_poses
        if fn is None:
            from .engine import rs_row_poses as fn
        return fn(*self._row_pose_args(p, rig, camvar, row))

    # ------------------------------------------------------------------ inertial factors + omega priors
    def _inertial(self, p: SessionProblem):
        nr = len(p.rig_ts_us)
        ts = p.rig_ts_us
        fvars = {k: [] for k in range(1, 4)}
        src = {k: ([], [], []) for k in range(1, 4)}
        for i in range(self.n_imu):
            for r in range(1, nr):
                if ts[r] - ts[r - 1] > K_MAX_INERTIAL_GAP_US:
                    continue
                calib = p.imu_var(r - 1, i)  # generatePreintegration: the previous rig's calibration
                if i == 0:
                    kind, v = 1, (calib, r - 1, r - 1, r, r, 0)
                else:
                    ep, en = p.imu_extr_var(r - 1, i), p.imu_extr_var(r, i)
                    if ep == en:
                        kind, v = 2, (calib, r - 1, r - 1, r - 1, r, r, r, ep, 0)
                    else:
                        kind, v = 3, (calib, r - 1, r - 1, r - 1, ep, r, r, r, en, 0)
                fvars[kind].append(v)
                for lst, val in zip(src[kind], (i, int(ts[r - 1]), int(ts[r]))):
                    lst.append(val)
        self.inertial = {}
        for k in (1, 2, 3):
            n = len(fvars[k])
            consts = np.zeros((n, kinds.factor_num_consts(k)))
            # placeholder preintegration (identity rotation, identity covariance) until the device
            # computes the real one after vb_finalize
            consts[:, 3] = 1.0
            consts[:, 10] = 0.1
            consts[:, 11 + 207:11 + 207 + 81] = np.eye(9).ravel()
            consts[:, 11 + 207 + 81:] = p.vars[6][np.array([v[0] for v in fvars[k]], np.int64)] if n else 0.0
            self.inertial[k] = (np.array(fvars[k], np.int32).reshape(n, kinds.factor_num_vars(k)), consts)
            p.preint_src[k] = tuple(np.array(a, dtype) for a, dtype in zip(src[k], (np.int32, np.int64, np.int64)))
        # addOmegaPriors (only with > 1 IMU): omegaAtEnd of every rig's preintegration, including the short
        # interval ahead of the first rig (and of rigs after a gap)
        om_v, om_c = [], []
        if self.n_imu > 1:
            for r in range(nr):
                for i in range(self.n_imu):
                    first = r == 0 or ts[r] - ts[r - 1] > K_MAX_INERTIAL_GAP_US
                    t0 = int(ts[r]) - K_SMALL_INTERVAL_FOR_OMEGA_US if first else int(ts[r - 1])
                    calib = p.vars[6][p.imu_var(r if first else r - 1, i)]
                    w = compensated_gyro_at_end(p.imu_streams[i], calib, t0, int(ts[r]))
                    om_v.append((r, -1 if i == 0 else p.imu_extr_var(r, i)))
                    om_c.append((*w, K_MULTI_IMU_OMEGA_PRIOR_STD))
        self.omega = (np.array(om_v, np.int32).reshape(-1, 2), np.array(om_c).reshape(-1, 4))

    # ------------------------------------------------------------------ random walks
    def _random_walks(self, p: SessionProblem):
        sd, m, s = self.sd, self.m, self.s
        nw, avg = self.nw, self.avg
        jac = ImuJacIndices(s.imu_calib_options)
        rw = {5: ([], []), 6: ([], []), 7: ([], []), 8: ([], [])}

        def dt(w):
            return (avg[w] - avg[w - 1]) * 1e-6
        for i in range(self.n_imu):   # addImuRWFactors (imu_model/RandomWalkCov.cpp imuCalibRandomWalkCov)
            nm = sd.imu_noise_models[m.slam_imu_to_factory[i]]
            for w in range(1, nw):
                q = np.zeros(jac.size)
                for name, val in (("aB", nm.accel_bias_rw_var), ("gB", nm.gyro_bias_rw_var),
                                  ("gS", nm.gyro_scale_rw_var), ("aS", nm.accel_scale_rw_var),
                                  ("aN", nm.accel_nonorth_rw_var)):
                    if getattr(jac, name) >= 0:
                        q[getattr(jac, name):getattr(jac, name) + 3] = dt(w) * val
                if jac.gN >= 0:
                    q[jac.gN:jac.gN + 6] = dt(w) * nm.gyro_nonorth_rw_var
                if jac.rT >= 0:
                    q[jac.rT] = nm.ref_imu_time_offset_rw_var * dt(w)
                if jac.gaT >= 0:
                    q[jac.gaT] = nm.gyro_accel_time_offset_rw_var * dt(w)
                q *= s.imu_rw_inflate
                c = np.zeros(23)
                c[:jac.size] = np.sqrt(1.0 / q)
                rw[5][0].append((i * nw + w - 1, i * nw + w))
                rw[5][1].append(c)
        for c_ in range(self.n_cam):  # addCamIntrinsicsRWFactors (camera_model/RandomWalkCov.cpp)
            for w in range(1, nw):
                cd = p.vars[4][c_ * nw + w]
                n_proj, n_dist = (4, 0) if cd[0] == 0 else (3, 12)
                nt = int(cd[7] != 0) + int(cd[8] != 0)
                q = np.concatenate([np.full(n_proj, K_CAM_PROJ_RW_VAR * dt(w)), np.full(n_dist, K_CAM_DIST_RW_VAR * dt(w)),
                                    np.full(nt, K_READOUT_RW_VAR * dt(w))]) * s.cam_intr_rw_inflate
                c = np.zeros(17)
                c[:len(q)] = np.sqrt(1.0 / q)
                rw[6][0].append((c_ * nw + w - 1, c_ * nw + w))
                rw[6][1].append(c)
        for i in range(1, self.n_imu):  # addImuExtrinsicsRWFactors (extrinsics_model/RandomWalkCov.cpp)
            nm = sd.imu_noise_models[m.slam_imu_to_factory[i]]
            for w in range(1, nw):
                q = np.concatenate([np.full(3, dt(w) * nm.imu_body_imu_pos_rw_var),
                                    np.full(3, dt(w) * nm.imu_body_imu_rot_rw_var)]) * s.imu_extr_rw_inflate
                rw[7][0].append(((i - 1) * nw + w - 1, (i - 1) * nw + w))
                rw[7][1].append(np.sqrt(1.0 / q))
        for c_ in range(self.n_cam):  # addCamExtrinsicsRWFactors
            for w in range(1, nw):
                q = np.concatenate([np.full(3, dt(w) * K_CAM_EXTR_RW_POS_VAR),
                                    np.full(3, dt(w) * K_CAM_EXTR_RW_ROT_VAR)]) * s.cam_extr_rw_inflate
                rw[8][0].append((c_ * nw + w - 1, c_ * nw + w))
                rw[8][1].append(np.sqrt(1.0 / q))
        self.rw = {k: (np.array(v, np.int32).reshape(-1, 2), np.array(c).reshape(-1, kinds.factor_num_consts(k)))
                   for k, (v, c) in rw.items()}

    # ------------------------------------------------------------------ factory priors
    def _factory_priors(self, p: SessionProblem):
        sd, m, s = self.sd, self.m, self.s
        nw = self.nw
        counts = np.bincount(p._rig_win, minlength=nw)   # rigs referencing each window's variable
        jac = ImuJacIndices(s.imu_calib_options)
        pri = {10: ([], []), 11: ([], []), 12: ([], []), 13: ([], [])}
        if s.cam_intr_factory_calib_inflate > 0:   # addCamIntrFactoryCalibPriors
            for c_ in range(self.n_cam):
                fc = sd.factory_calib.cameras[m.slam_cam_to_factory[c_]]
                prior = fc.camera_data(False, False)
                for w in range(nw):
                    cd = p.vars[4][c_ * nw + w]
                    if abs(prior[9] - cd[9]) / prior[9] >= 0.1:   # kFocalLEngthMaxRelError
                        raise ValueError(f"Camera n. {c_}: factory calibration prior params are very different "
                                         "from online calibration params (incorrectly adapted resolution?)")
                    n_proj, n_dist = (4, 0) if cd[0] == 0 else (3, 12)
                    std = [K_CAM_PROJ_TURNON_STD] * n_proj + [K_CAM_DIST_TURNON_STD] * n_dist
                    if cd[7] != 0:
                        std.append(K_CAM_RO_TURNON_STD)
                    if cd[8] != 0:
                        std.append(K_CAM_OFF_TURNON_STD)
                    if len(std) != n_proj + n_dist:  # addCamIntrinsicsPrior: prior / variable tangent dims
                        raise ValueError("camera intrinsics prior: tangent size differs from the variable's "
                                         "(estimated readout / offset with a factory prior, PriorFactor.cpp:118-120)")
                    std = np.array(std) * s.cam_intr_factory_calib_inflate
                    H = counts[w] / std ** 2
                    c = np.zeros(41)
                    c[:24] = prior
                    c[24:24 + len(H)] = H
                    pri[11][0].append((c_ * nw + w,))
                    pri[11][1].append(c)
        if s.cam_extr_factory_calib_inflate > 0:   # addCamExtrFactoryCalibPriors (rotation std converted
            for c_ in range(self.n_cam):            # from degrees once more, as the reference does)
                T = sd.factory_calib.T_cam_bodyimu[m.slam_cam_to_factory[c_]]
                std = np.array([K_CAM_EXTR_POS_TURNON_STD] * 3 + [K_CAM_EXTR_ROT_TURNON_STD * math.pi / 180] * 3)
                std = std * s.cam_extr_factory_calib_inflate
                for w in range(nw):
                    pri[12][0].append((c_ * nw + w,))
                    pri[12][1].append(np.concatenate([T, counts[w] / std ** 2]))
        if s.imu_extr_factory_calib_inflate > 0 and self.n_imu > 1:   # addImuExtrFactoryCalibPriors
            for i in range(1, self.n_imu):
                fi = m.slam_imu_to_factory[i]
                T = sd.factory_calib.T_imu_bodyimu[fi]
                nm = sd.imu_noise_models[fi]
                std = np.array([nm.imu_body_imu_turnon_pos_std] * 3 + [nm.imu_body_imu_turnon_rot_std] * 3)
                std = std * s.imu_extr_factory_calib_inflate
                for w in range(nw):
                    pri[13][0].append(((i - 1) * nw + w,))
                    pri[13][1].append(np.concatenate([T, counts[w] / std ** 2]))
        if s.imu_factory_calib_inflate > 0:   # addImuFactoryCalibPriors (imuCalibTurnonStdDev)
            for i in range(self.n_imu):
                fi = m.slam_imu_to_factory[i]
                nm = sd.imu_noise_models[fi]
                std = np.zeros(jac.size)
                for name, val in (("gB", nm.gyro_bias_turnon_std), ("aB", nm.accel_bias_turnon_std),
                                  ("gS", nm.gyro_scale_turnon_std), ("aS", nm.accel_scale_turnon_std),
                                  ("aN", nm.accel_nonorth_turnon_std)):
                    if getattr(jac, name) >= 0:
                        std[getattr(jac, name):getattr(jac, name) + 3] = val
                if jac.gN >= 0:
                    std[jac.gN:jac.gN + 6] = nm.gyro_nonorth_turnon_std
                if jac.rT >= 0:
                    std[jac.rT] = nm.ref_imu_time_offset_turnon_std
                if jac.gaT >= 0:
                    std[jac.gaT] = nm.gyro_accel_time_offset_turnon_std
                std = std * s.imu_factory_calib_inflate
                for w in range(nw):
                    c = np.zeros(55)
                    c[:32] = sd.factory_calib.imu_models[fi]
                    c[32:32 + jac.size] = counts[w] / std ** 2
                    pri[10][0].append((i * nw + w,))
                    pri[10][1].append(c)
        self.priors = {k: (np.array(v, np.int32).reshape(-1, 1), np.array(c).reshape(-1, kinds.factor_num_consts(k)))
                       for k, (v, c) in pri.items()}

    # ------------------------------------------------------------------ assembly
    def problem(self) -> SessionProblem:
        p = self.build()
        p.fvars, p.fivals, p.fconsts = [], [], []
        per_kind = {0: (self.visual[0], self.visual[1], self.visual[2]), 4: (*self.omega,)}
        for k in (1, 2, 3):
            per_kind[k] = self.inertial[k]
        per_kind.update(self.rw)
        per_kind.update(self.priors)
        for k in range(kinds.NUM_FACTOR_KINDS):
            nv, nc = kinds.factor_num_vars(k), kinds.factor_num_consts(k)
            if k not in per_kind:
                p.fvars.append(np.zeros((0, nv), np.int32))
                p.fivals.append(np.zeros(0, np.int32))
                p.fconsts.append(np.zeros((0, nc)))
                continue
            t = per_kind[k]
            fv, fc = (t[0], t[2]) if k == 0 else (t[0], t[1])
            fi = t[1] if k == 0 else np.full(len(fv), -1, np.int32)
            p.fvars.append(np.ascontiguousarray(fv, np.int32).reshape(-1, nv))
            p.fivals.append(np.ascontiguousarray(fi, np.int32))
            p.fconsts.append(np.ascontiguousarray(fc, np.float64).reshape(-1, nc))
        return p


def build_problem(sd: SessionData, matcher: Matcher | None = None, settings: InitSettings | None = None,
                  row_poses=None) -> SessionProblem:
    """SessionData -> SessionProblem (ark_vi_ba main_AriaKit_ViBa.cpp:49-63).  row_poses: the
    T_bodyImu_world_atImageRow provider of the triangulation (default: the device, vb_rs_row_poses)."""
    return SessionAdapter(sd, matcher or Matcher.build(sd), settings, row_poses).problem()


def load_into(engine, p: SessionProblem, finalize: bool = True, recompute_preint: bool | None = None):
    """Feed a session problem to an engine: variables, the IMU streams, the rolling-shutter intervals
    (rebuilt from the IMU-0 stream by the engine, updateRollingShutterData), the factors, the
    preintegration sources; after vb_finalize the engine computes every preintegration
    (regenerateAllPreintegrationsFromImuMeasurements) and the rolling-shutter tables."""
    for k in range(kinds.NUM_VAR_KINDS):
        engine.set_vars(k, p.vars[k], p.const[k])
    s0 = p.imu_streams[0]
    engine.set_imu_measurements(s0.timestamp_ns, s0.gyro, s0.accel)
    if p.rs_mid is not None and len(p.rs_mid):
        engine.set_rs_rigs(p.rs_mid, p.rs_half, p.rs_calib, 0)
    for i, st in enumerate(p.imu_streams):
        if i > 0:
            engine.set_imu_stream(i, st.timestamp_ns, st.gyro, st.accel)
        engine.set_imu_noise(i, *p.imu_noise[i])
    for f in range(kinds.NUM_FACTOR_KINDS):
        if len(p.fivals[f]):
            engine.add_factors(f, p.fvars[f], p.fivals[f], p.fconsts[f])
    for k in (1, 2, 3):
        if len(p.fvars[k]):
            engine.set_preint_sources(k, *p.preint_src[k])
    if recompute_preint:
        engine.set_recompute_preint(True)
    engine.rs_device = p.rs_mid is not None and len(p.rs_mid) > 0
    if finalize:
        engine.finalize()
        if engine.rs_device:
            engine.update_rs_tables()
        if any(len(p.fvars[k]) for k in (1, 2, 3)):
            engine.update_preintegrations()
    return engine


def save_outputs(out_dir: str, engine, p: SessionProblem, sd: SessionData):
    """ark_vi_ba's outputs (main_AriaKit_ViBa.cpp:122-130) from an engine's current variables:
    online_calibration.jsonl, open_loop_framerate_trajectory.csv, closed_loop_framerate_trajectory.csv."""
    import os

    from . import session as S
    os.makedirs(out_dir, exist_ok=True)
    v = [engine.get_vars(k) for k in range(kinds.NUM_VAR_KINDS)]
    nr = len(p.rig_ts_us)
    cams = [[v[4][p.cam_var(r, s)] for s in range(p.n_cam)] for r in range(nr)]
    extr = [[v[5][p.cam_var(r, s)] for s in range(p.n_cam)] for r in range(nr)]
    imus = [[v[6][p.imu_var(r, s)] for s in range(p.n_imu)] for r in range(nr)]
    iext = [[None] + [v[7][p.imu_extr_var(r, s)] for s in range(1, p.n_imu)] for r in range(nr)]
    S.save_online_calibration(os.path.join(out_dir, "online_calibration.jsonl"), sd, p.rig_pose_index, cams, extr,
                              imus, iext)
    ps = sd.inertial_poses
    idx = p.rig_pose_index
    rigs = S.InertialPoses(ps.T_w_imu[idx], ps.v_w[idx], ps.omega_bodyimu[idx], ps.timestamp_us[idx],
                           ps.utc_timestamp_ns[idx], ps.quality[idx], [ps.uid[i] for i in idx])
    rv, g = (v[1], v[2], v[3]), v[8][0, :3]
    S.write_open_loop_trajectory(os.path.join(out_dir, "open_loop_framerate_trajectory.csv"), rigs, rv,
                                 sd.T_bodyimu_device, g)
    S.write_closed_loop_trajectory(os.path.join(out_dir, "closed_loop_framerate_trajectory.csv"), rigs, rv,
                                   sd.T_bodyimu_device, g)


def run_session(in_dir: str, out_dir: str | None = None, engine_factory=None, settings: InitSettings | None = None,
                optimizer_settings=None, refine: bool = True, log=print):
    """ark_vi_ba (interfaces/ark/main_AriaKit_ViBa.cpp:32-133) on a session folder: load, build indices,
    build the problem, rolling-shutter tables, refinePoints, Optimizer::optimize (with the per-iteration
    rolling-shutter rebuild and, under settings.recompute_preint, the preintegration recompute of the
    preStepCallback), then the three output files.  engine_factory(problem) -> engine (default: the HIP
    engine).  Returns (engine, problem, summary)."""
    from .engine import HipEngine, Settings
    s = settings or InitSettings()
    sd = SessionData.load(in_dir, load_imu=True)
    m = Matcher.build(sd)
    p = SessionAdapter(sd, m, s).problem()
    if log:
        log(f"[ark] {p.summary()}; {p.triangulated} of {p.tried_tracks} tracks triangulated")
    if engine_factory is None:
        def engine_factory(q):
            return HipEngine(reproj_loss=q.reproj_loss, imu_loss=q.imu_loss, imu_calib_options=q.imu_calib_options)
    e = load_into(engine_factory(p), p, recompute_preint=s.recompute_preint)
    if refine:
        (c0, c1), _ = e.refine_points()
        if log:
            log(f"[ark] refinePoints: visual cost {c0:.6g} -> {c1:.6g}")
    summary = e.optimize(optimizer_settings or Settings.default())
    if log:
        log(f"[ark] optimize: {summary.initial_cost:.6g} -> {summary.final_cost:.6g} in {summary.num_iterations} iterations")
    if out_dir:
        save_outputs(out_dir, e, p, sd)
    return e, p, summary
