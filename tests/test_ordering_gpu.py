"""The reduced system's nested-dissection order (api.hip finalize): the cut at the thinnest
separator within +-5% of the median (default) against the plain median cut with left separators
(VIBA_ND_CUTWIN=0 VIBA_ND_SEPRIGHT=0).  Both are valid Cholesky orders: the LM step is the same to
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
    st_med, mr_med, s_med = _run({"VIBA_ND_CUTWIN": "0", "VIBA_ND_SEPRIGHT": "0"})
    assert st_thin[3] >= st_thin[2] and st_med[3] >= st_med[2]  # reduced order incl. tile padding
    assert st_thin[6] <= st_med[6], (st_thin[6], st_med[6])  # tile-pair contributions per factorization
    assert abs(mr_thin - mr_med) <= 1e-9 * abs(mr_med)
    for a, b in zip(s_thin, s_med):
        assert rel(np.asarray(a), np.asarray(b)) < 1e-8
