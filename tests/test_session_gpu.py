"""The committed reference-format session folder (tests/golden/session_small) end to end
on the GPU: SessionData.load -> Matcher -> SessionAdapter -> the HIP engine through the C-ABI
(preintegrations and rolling-shutter tables computed on the device) against the CPU oracle on the same
folder, then ark_vi_ba's pipeline (refinePoints, optimize, the three output files) on both engines."""
from __future__ import annotations

import os

import numpy as np
import pytest

from visual_inertial_bundle_adjustment_amd import adapter, session
from visual_inertial_bundle_adjustment_amd.engine import HipEngine, Settings

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "session_small")


def _engines(q):
    from oracle.refcpu import RefEngine
    kw = dict(reproj_loss=q.reproj_loss, imu_loss=q.imu_loss, imu_calib_options=q.imu_calib_options)
    return adapter.load_into(HipEngine(**kw), q), adapter.load_into(RefEngine(**kw), q)


@pytest.mark.parametrize("folder", ["golden", "generated"])
def test_rs_row_poses_and_triangulation_match_oracle(folder, tmp_path):
    """T_bodyImu_world_atImageRow on the device (vb_rs_row_poses: tables rebuilt from the IMU stream,
    rs_row_pose_kernel) against the oracle's (RollingShutterData::compute + getEstimate on the host), on the
    adapter's own inputs: poses within 1e-12; and the problems the adapter builds from the two are the
    same -- identical accepted tracks and visual factors (refine-2 inlier sets), points within 1e-9."""
    from oracle.refcpu import rs_row_poses as ref_row_poses
    from visual_inertial_bundle_adjustment_amd import synth
    from visual_inertial_bundle_adjustment_amd.engine import rs_row_poses
    if folder == "golden":
        d = GOLDEN
    else:
        d = str(tmp_path / "s")
        synth.write_session(synth.generate(synth.config("miniB", n_kf=80, n_lm=400)), d)
    sd = session.SessionData.load(d)
    a = adapter.SessionAdapter(sd, session.Matcher.build(sd))          # the device provider (default)
    q = a.problem()
    b = adapter.SessionAdapter(sd, session.Matcher.build(sd), None, ref_row_poses)
    qr = b.problem()
    args = a._row_pose_args(q, *a.row_pose_inputs)
    dev, ref = rs_row_poses(*args), ref_row_poses(*args)
    assert np.abs(dev - ref).max() < 1e-12
    assert np.array_equal(a.triangulation["ok"], b.triangulation["ok"])
    assert np.array_equal(a.triangulation["inliers"], b.triangulation["inliers"])
    assert np.abs(q.vars[0] - qr.vars[0]).max() < 1e-9
    assert np.array_equal(q.fvars[0], qr.fvars[0]) and np.array_equal(q.fconsts[0], qr.fconsts[0])


def test_rs_row_poses_errors():
    """the reference throws for a row time outside the table (getEstimate) and aborts for a rolling-shutter
    camera on a rig without one (findOrDie): VB_E_RANGE / VB_E_ARG"""
    from visual_inertial_bundle_adjustment_amd.engine import VbError, rs_row_poses
    sd = session.SessionData.load(GOLDEN)
    a = adapter.SessionAdapter(sd, session.Matcher.build(sd))
    q = a.problem()
    rig, camvar, row = a.row_pose_inputs
    args = list(a._row_pose_args(q, rig, camvar, row))
    rs_obs = np.flatnonzero([q.vars[4][c][4] != 0 for c in camvar])[:1]
    bad_row = row.copy()
    bad_row[rs_obs] = 1e9                                   # far past the readout: outside the table
    with pytest.raises(VbError) as ex:
        rs_row_poses(*args[:13], bad_row)
    assert ex.value.code == -5
    no_table = np.full_like(args[9], -1)
    with pytest.raises(VbError) as ex:
        rs_row_poses(*args[:9], no_table, *args[10:])
    assert ex.value.code == -1


def test_session_folder_step_matches_oracle():
    from parity_util import gradient_entry_errors, one_step, rel
    q = adapter.build_problem(session.SessionData.load(GOLDEN))
    g, r = _engines(q)
    # the device's preintegrations of every inertial row against the oracle's
    for k in (1, 2, 3):
        for row in range(0, len(q.fvars[k]), 7):
            assert rel(g.get_factor_consts(k, row)[:299], r.get_factor_consts(k, row)[:299]) < 1e-10
    og, orf = one_step(g), one_step(r)
    assert abs(og["cost0"] - orf["cost0"]) <= 1e-10 * abs(orf["cost0"])
    assert abs(og["model_red"] - orf["model_red"]) <= 1e-9 * abs(orf["model_red"])
    assert abs(og["cost1"] - orf["cost1"]) <= 1e-9 * abs(orf["cost1"])
    assert og["stats1"] == orf["stats1"]
    # per entry, against the sum of the magnitudes of the terms the entry adds up (the oracle's
    # ref_abs_gradient at x0): the triangulated points start near their optimum, so their gradients are
    # cancellation residues of terms many orders larger, and a tolerance relative to the largest entry
    # (1e-9 here until round 4) cannot tell summation order from an assembly error.  The bound: the
    # rolling-shutter time columns are forward differences with eps = 1e-6 (VisualFactor.cpp), so a term's
    # own round-off reaches ~2^-52 / 1e-6 = 2e-10 of it; measured 7.5e-12 (r05)
    worst = gradient_entry_errors(og["grad"], orf["grad"], r)
    print('gradient entry errors / term magnitudes:', worst)
    assert max(worst.values()) < 1e-10, worst
    for a, b in zip(og["step"], orf["step"]):
        if b.size:
            assert rel(a, b) < 1e-8
    stored = np.load(os.path.join(HERE, "golden", "session_small.npz"))
    assert abs(og["cost0"] - stored["cost0"]) <= 1e-9 * abs(stored["cost0"])


def test_session_pipeline_matches_oracle(tmp_path):
    """run_session (main_AriaKit_ViBa.cpp:49-130) with the HIP engine and with the oracle: same LM
    trajectory, and output files that agree."""
    from oracle.refcpu import RefEngine
    from parity_util import rel
    st = Settings.default(max_num_iterations=8)
    eg, q, sg = adapter.run_session(GOLDEN, str(tmp_path / "gpu"), optimizer_settings=st, log=None)
    er, _, sr = adapter.run_session(GOLDEN, str(tmp_path / "cpu"), optimizer_settings=st, log=None,
                                    engine_factory=lambda p: RefEngine(reproj_loss=p.reproj_loss, imu_loss=p.imu_loss,
                                                                       imu_calib_options=p.imu_calib_options))
    assert sg.num_iterations == sr.num_iterations
    assert abs(sg.initial_cost - sr.initial_cost) <= 1e-10 * sr.initial_cost
    assert abs(sg.final_cost - sr.final_cost) <= 1e-9 * sr.final_cost
    for k in range(1, 8):
        a, b = eg.get_vars(k), er.get_vars(k)
        if len(b):
            assert rel(a, b) < 1e-7, k
    cg = session.read_online_calibration(tmp_path / "gpu" / "online_calibration.jsonl")
    cc = session.read_online_calibration(tmp_path / "cpu" / "online_calibration.jsonl")
    assert len(cg) == len(cc) == len(q.rig_ts_us)
    for (t1, _, c1, i1), (t2, _, c2, i2) in zip(cg, cc):
        assert t1 == t2
        for a, b in zip(c1, c2):
            assert rel(a.params, b.params) < 1e-7
        for a, b in zip(i1, i2):
            assert rel(a.model, b.model) < 1e-7
    for name in ("open_loop_framerate_trajectory.csv", "closed_loop_framerate_trajectory.csv"):
        a = open(tmp_path / "gpu" / name).read().splitlines()
        b = open(tmp_path / "cpu" / name).read().splitlines()
        assert a[0] == b[0] and len(a) == len(b) == len(q.rig_ts_us) + 1
        va = np.array([[float(x) for x in line.split(",")[3:19]] for line in a[1:]])
        vb = np.array([[float(x) for x in line.split(",")[3:19]] for line in b[1:]])
        assert np.allclose(va, vb, rtol=2e-5, atol=2e-6)   # 6 significant digits per value
