"""The LM controller's variable-tolerance test (Optimizer.cpp:1014-1018) on a rescaled iteration.

`toleranceHit` reads ratioS2Vn2 from the FULL step's applyStep (Optimizer.cpp:886); the rescaled
attempts' applyStep calls (:927, :972) discard their ratios.  Every controller restates this: the oracle
(oracle/refcpu.cpp ref_optimize), vb_optimize (api.hip) and the Python controller of the multi-process
path (distributed.ShardedOptimizer).  The case only shows when a rescaled iteration's full step is above
`variables_tolerance` and its scaled step below it, with `stop_if_no_improvement_for=1` so that the
tolerance decides the iteration count: `variables_tolerance` is placed between the two, on the first
iteration, so a controller reading the scaled step's ratio stops after one iteration and one reading the
full step's goes on.  (Until round 5 the oracle read the scaled one.)
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from parity_util import make, rel
from visual_inertial_bundle_adjustment_amd.engine import Settings
from visual_inertial_bundle_adjustment_amd.kinds import NUM_VAR_KINDS

LAM0 = 1e-5  # Settings.default().damping: the first iteration's damping


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def full_step_rms(engine_cls, which):
    """ratioS2Vn2 of the first iteration's full step (Optimizer.cpp:807-886 by the engine's primitives)."""
    e, _ = make(engine_cls, which)
    e.linearize(True, False)
    e.damp_factor_solve(LAM0)
    e.backup()
    r = e.apply_step(0)
    e.restore()
    return r[1]


def tolerance_settings(full_rms, max_its=6):
    """Every full step misses min_relative_cost_reduction (so every iteration rescales, and the scaled
    step's RMS ratio is applied x the full one's, applied < 1); variables_tolerance just under the first
    full step's ratio; the cost tolerances off; stop at the first iteration that hits a tolerance."""
    return Settings.default(max_num_iterations=max_its, min_relative_cost_reduction=1.02,
                            variables_tolerance=0.999 * full_rms, relative_cost_tolerance=-1e300,
                            absolute_cost_tolerance=-1e300, stop_if_no_improvement_for=1,
                            distance_from_troubled_iteration=0)


def _py_worker(rank, world, port, which, settings_bytes, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    import torch.distributed as dist
    from oracle.refcpu import RefEngine
    from parity_util import make
    from visual_inertial_bundle_adjustment_amd.distributed import ShardComm, ShardedOptimizer
    from visual_inertial_bundle_adjustment_amd.engine import Settings

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    e, _ = make(RefEngine, which)
    n_pts = (e.total_order() - e.reduced_order()) // 3
    e.set_landmark_shard(0, n_pts, True)
    opt = ShardedOptimizer(e, ShardComm(rank, world, None))
    # record every box-plus's RMS ratio (full step first, then the rescaled attempts)
    applied = []
    inner = e.apply_step_raw
    n = max(1, e.num_params())

    def apply_step_raw(which=0):
        r = inner(which)
        applied.append((which, r[0], (r[1] / n) ** 0.5, r[2] / n))
        return r
    e.apply_step_raw = apply_step_raw
    s = opt.optimize(Settings.from_buffer_copy(settings_bytes))
    np.savez(os.path.join(out_dir, "py.npz"), iters=s.num_iterations, rescaled=s.num_rescaled,
             final=s.final_cost, applied=np.array(applied),
             **{f"v{k}": e.get_vars(k) for k in range(1, NUM_VAR_KINDS - 1)})
    dist.destroy_process_group()


@pytest.mark.parametrize("which", ["A"])
def test_variable_tolerance_reads_full_step_ratio_cpu(which, tmp_path):
    """The Python controller (one gloo rank over the oracle's primitives; its loop restates
    Optimizer.cpp:800-1097 independently of ref_optimize) and ref_optimize give the same trajectory, and
    the variable tolerance did not stop the first (rescaled) iteration."""
    from oracle.refcpu import RefEngine
    full = full_step_rms(RefEngine, which)
    s = tolerance_settings(full)
    mp.spawn(_py_worker, args=(1, _free_port(), which, bytes(s), str(tmp_path)), nprocs=1, join=True)
    py = dict(np.load(tmp_path / "py.npz"))
    # the case is the discriminating one: iteration 0's full step is above the tolerance, its first
    # rescaled attempt below it
    ap = py["applied"]
    assert ap[0][0] == 0 and abs(ap[0][2] - full) <= 1e-12 * full and ap[0][2] >= s.variables_tolerance
    assert ap[1][0] == 0 and ap[1][2] < s.variables_tolerance
    e, _ = make(RefEngine, which)
    so = e.optimize(s)
    assert so.num_iterations >= 2  # the scaled step's ratio would have stopped it after one
    assert int(py["iters"]) == so.num_iterations
    assert int(py["rescaled"]) == so.num_rescaled == so.num_iterations
    assert abs(float(py["final"]) - so.final_cost) <= 1e-11 * so.final_cost
    for k in range(1, NUM_VAR_KINDS - 1):
        ref = e.get_vars(k)
        if len(ref):
            assert rel(py[f"v{k}"], ref) < 1e-9, k


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["A", "miniB"])
def test_variable_tolerance_reads_full_step_ratio_gpu(which):
    """vb_optimize against the oracle on the same discriminating settings: same iteration count (≥ 2),
    rescaled count, final cost and variables."""
    from oracle.refcpu import RefEngine
    from visual_inertial_bundle_adjustment_amd.engine import HipEngine
    full = full_step_rms(RefEngine, which)
    assert abs(full_step_rms(HipEngine, which) - full) <= 1e-8 * full
    s = tolerance_settings(full)
    g, _ = make(HipEngine, which)
    r, _ = make(RefEngine, which)
    sg, sr = g.optimize(s), r.optimize(s)
    assert sr.num_iterations >= 2
    assert sg.num_iterations == sr.num_iterations and sg.num_rescaled == sr.num_rescaled
    assert abs(sg.final_cost - sr.final_cost) <= 1e-9 * sr.final_cost
    for k in range(1, NUM_VAR_KINDS - 1):
        ref = r.get_vars(k)
        if len(ref):
            assert rel(g.get_vars(k), ref) < 1e-7, k
