"""The reduced system's nested-dissection order (api.hip finalize): the cut at the thinnest
separator within +-5% of the median (default) against the plain median cut with left separators
(VIBA_ND_CUTWIN=0).  Both are valid Cholesky orders: the LM step is the same to
round-off; the thin cut needs fewer tile contributions.  The variables are read at vb_finalize."""
from __future__ import annotations

import os

import numpy as np
import pytest

from parity_util import make, rel

pytestmark = pytest.mark.gpu


def _run(env):
    from visual_inertial_bundle_adjustment_amd.engine import HipEngine
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        e, p = make(HipEngine, "B")
        st = e.problem_stats()
        e.linearize(True, False)
        mr = e.damp_factor_solve(1e-4)
        step = [e.get_step(k) for k in (1, 2, 4)]
        e.close()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return st, mr, step


def test_thin_separator_order_same_step_fewer_contributions():
    st_thin, mr_thin, s_thin = _run({})
    st_med, mr_med, s_med = _run({"VIBA_ND_CUTWIN": "0"})
    assert st_thin[3] >= st_thin[2] and st_med[3] >= st_med[2]  # reduced order incl. tile padding
    assert st_thin[6] <= st_med[6], (st_thin[6], st_med[6])  # tile-pair contributions per factorization
    assert abs(mr_thin - mr_med) <= 1e-9 * abs(mr_med)
    for a, b in zip(s_thin, s_med):
        assert rel(np.asarray(a), np.asarray(b)) < 1e-8


def test_stats_knob_prints_and_changes_nothing(capfd):
    """VIBA_STATS=1 (diagnostics only: the supernode streams' contributions and the Schur work's compact
    widths, MFMA padding and gathered bytes, printed at vb_finalize) leaves the arithmetic alone."""
    st0, mr0, s0 = _run({})
    capfd.readouterr()
    st1, mr1, s1 = _run({"VIBA_STATS": "1"})
    err = capfd.readouterr().err
    assert "[schur stats]" in err and "[factor stats]" in err, err[-2000:]
    # (same order and schedule; fp64 atomics leave run-to-run round-off, DESIGN.md §2: ~1e-13)
    assert tuple(st0) == tuple(st1) and abs(mr0 - mr1) <= 1e-11 * abs(mr0)
    for a, b in zip(s0, s1):
        assert rel(np.asarray(a), np.asarray(b)) < 1e-10


def test_time_order_leaf_same_step_fewer_contributions_more_levels():
    """A leaf larger than the system (VIBA_ND_LEAF, what bench.py's banded count sets): one part in time
    order, the band the reference's solver sees. Same step. The band needs fewer tile contributions (config B:
    69k against the dissection's 132k) but is one long chain of dependent columns: the dissection buys its
    level parallelism with flops."""
    st_nd, mr_nd, s_nd = _run({})
    st_tm, mr_tm, s_tm = _run({"VIBA_ND_LEAF": str(1 << 62)})
    assert st_tm[6] < st_nd[6], (st_tm[6], st_nd[6])  # tile-pair contributions per factorization
    assert st_tm[10] > st_nd[10], (st_tm[10], st_nd[10])  # elimination levels
    assert abs(mr_tm - mr_nd) <= 1e-9 * abs(mr_nd)
    for a, b in zip(s_tm, s_nd):
        assert rel(np.asarray(a), np.asarray(b)) < 1e-8
