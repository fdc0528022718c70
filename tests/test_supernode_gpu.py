"""The two-column supernode factorization (VIBA_SUPERNODE=1 at handle creation; api.hip SnSched,
solver.hip snpotrf_kernel / sntrsm_kernel) against the oracle and against the column schedule.

A pair (J, J + 1) -- J + 1 the parent of J, J's other rows all rows of J + 1 -- is factored as one
128-wide diagonal block and its rows in one pass, so the schedule has about half the levels.  The
arithmetic is the same Cholesky in another association order: steps agree with the column schedule and
the oracle to round-off (stated per test)."""
from __future__ import annotations

import numpy as np
import pytest

from oracle.refcpu import RefEngine
from parity_util import make, one_step, rel
from visual_inertial_bundle_adjustment_amd import synth
from visual_inertial_bundle_adjustment_amd.kinds import NUM_VAR_KINDS, VAR_NAMES

pytestmark = pytest.mark.gpu


def _hip(p, sn: bool, streams: int | None = None):
    from visual_inertial_bundle_adjustment_amd.engine import HipEngine
    with pytest.MonkeyPatch.context() as mp:
        mp.setenv("VIBA_SUPERNODE", "1" if sn else "0")  # read when the handle is created
        if streams is not None:
            mp.setenv("VIBA_SN_STREAMS", str(streams))
        e = HipEngine(imu_calib_options=p.imu_calib_options)
    synth.load_into(e, p)
    return e


@pytest.mark.parametrize("which", ["A", "miniB", "B"])
def test_supernode_step_matches_oracle_and_column_schedule(which):
    from test_parity_gpu import assert_step_parity
    p = synth.generate(synth.config(which))
    g, c = _hip(p, True), _hip(p, False)
    lv, contrib, nsup, ntwo = g.factor_schedule_stats()
    lv0, contrib0, _, ntwo0 = c.factor_schedule_stats()
    print(f"{which}: supernode schedule {lv} levels ({ntwo} of {nsup} supernodes two-column), fan-in "
          f"contributions {contrib}; column schedule {lv0} levels, {contrib0}")
    assert ntwo0 == 0 and lv <= lv0 and contrib <= contrib0
    if which != "A":
        assert ntwo > 0 and lv < lv0
    r = RefEngine(imu_calib_options=p.imu_calib_options)
    synth.load_into(r, p)
    og, oc = one_step(g), one_step(c)
    assert_step_parity(og, one_step(r))
    for k in range(NUM_VAR_KINDS - 1):
        if oc["step"][k].size:
            assert rel(og["step"][k], oc["step"][k]) < 1e-9, VAR_NAMES[k]
            assert rel(og["substep"][k], oc["substep"][k]) < 1e-8, VAR_NAMES[k]


def test_supernode_optimize_matches_oracle():
    p = synth.generate(synth.config("miniB"))
    g = _hip(p, True)
    r = RefEngine(imu_calib_options=p.imu_calib_options)
    synth.load_into(r, p)
    from visual_inertial_bundle_adjustment_amd.engine import Settings
    s = Settings.default(max_num_iterations=10)
    sg, sr = g.optimize(s), r.optimize(s)
    assert sg.num_iterations == sr.num_iterations and sg.num_rescaled == sr.num_rescaled
    assert abs(sg.final_cost - sr.final_cost) <= 1e-9 * sr.final_cost
    for k in range(NUM_VAR_KINDS - 1):
        if len(r.get_vars(k)):
            assert rel(g.get_vars(k), r.get_vars(k)) < 1e-7, VAR_NAMES[k]


def test_supernode_covariances_match_column_schedule():
    """the selected inversion consumes the factor whichever schedule produced it"""
    p = synth.generate(synth.config("miniB"))
    g, c = _hip(p, True), _hip(p, False)
    blocks = [[(1, 0), (2, 0)], [(1, 5)], [(2, 3), (1, 60)], [(4, 0)]]
    (a, _), (b, _) = g.compute_covariances(blocks), c.compute_covariances(blocks)
    for x, y in zip(a, b):
        assert rel(x, y) < 1e-9


@pytest.mark.parametrize("streams", [2, 3, 4])
def test_supernode_streams_match_one_stream(streams):
    """the schedule's independent subtrees on `streams` streams (api.hip factorSeqSn: forked from the main
    stream, cross-stream waits where a separator's children run elsewhere) factor the same matrix as one
    stream: the step of one LM iteration and a 6-iteration trajectory on config B agree to round-off (the
    fp64 atomics of the fused forward solve add in another order), and against the oracle"""
    from test_parity_gpu import assert_step_parity
    from visual_inertial_bundle_adjustment_amd.engine import Settings
    p = synth.generate(synth.config("B"))
    g, c = _hip(p, True, streams), _hip(p, True, 1)
    og, oc = one_step(g), one_step(c)
    for k in range(NUM_VAR_KINDS - 1):
        if oc["step"][k].size:
            assert rel(og["step"][k], oc["step"][k]) < 1e-9, VAR_NAMES[k]
    r = RefEngine(imu_calib_options=p.imu_calib_options)
    synth.load_into(r, p)
    assert_step_parity(og, one_step(r))
    g2, c2 = _hip(p, True, streams), _hip(p, True, 1)
    s = Settings.default(max_num_iterations=6)
    sg, sc = g2.optimize(s), c2.optimize(s)
    assert sg.num_iterations == sc.num_iterations and sg.num_rescaled == sc.num_rescaled
    assert abs(sg.final_cost - sc.final_cost) <= 1e-10 * sc.final_cost
