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


def test_session_folder_step_matches_oracle():
    from parity_util import one_step, rel
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
    for a, b in zip(og["grad"], orf["grad"]):
        if b.size:
            assert rel(a, b) < 1e-10
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
