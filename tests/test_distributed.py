"""Multi-device controller (visual_inertial_bundle_adjustment_amd/distributed.py) on CPU: two gloo
ranks, each owning half of the landmarks, driving the oracle's shard primitives, must reproduce the
single-process oracle's Optimizer::optimize (same iterations, same costs and variables up to
summation order)."""
from __future__ import annotations

import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from visual_inertial_bundle_adjustment_amd.engine import Settings


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _settings(its):
    return Settings.default(max_num_iterations=its)


def _worker(rank, world, port, which, its, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    import torch.distributed as dist
    from oracle.refcpu import RefEngine
    from parity_util import make
    from visual_inertial_bundle_adjustment_amd.distributed import ShardComm, ShardedOptimizer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    e, p = make(RefEngine, which)
    n_pts = (e.total_order() - e.reduced_order()) // 3
    cuts = [n_pts * r // world for r in range(world + 1)]
    e.set_landmark_shard(cuts[rank], cuts[rank + 1], rank == 0)
    opt = ShardedOptimizer(e, ShardComm(rank, world, None))
    s = opt.optimize(_settings(its))
    f = e.lib.ref_var_param
    f.restype, f.argtypes = C.c_int64, [C.c_void_p, C.c_int, C.c_int64]
    pts = e.get_vars(0)
    own = np.array([cuts[rank] <= f(e.h, 0, k) < cuts[rank + 1] for k in range(len(pts))])
    res = {"iters": s.num_iterations, "initial": s.initial_cost, "final": s.final_cost, "own": own, "pts": pts,
           "reads": np.array(opt.reads_per_iteration)}
    for k in range(1, 8):
        res[f"v{k}"] = e.get_vars(k)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    dist.destroy_process_group()


@pytest.mark.parametrize("which,its", [("A", 50), ("miniB", 6)])
def test_two_shards_match_single_process(which, its, tmp_path):
    from oracle.refcpu import RefEngine
    from parity_util import make, rel
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), which, its, str(tmp_path)), nprocs=world, join=True)
    r = [dict(np.load(tmp_path / f"rank{k}.npz")) for k in range(world)]
    e, _ = make(RefEngine, which)
    s = e.optimize(_settings(its))
    for k in range(world):
        assert int(r[k]["iters"]) == s.num_iterations
        assert abs(float(r[k]["initial"]) - s.initial_cost) <= 1e-11 * s.initial_cost
        assert abs(float(r[k]["final"]) - s.final_cost) <= 1e-9 * s.final_cost
    # the two partial Schur complements are summed on the root, so S differs from the single-process
    # sum by round-off; config A's reduced system is ill-conditioned at small damping (test_pcg.py) and
    # 50 LM iterations amplify that to ~2e-8 relative in the variables
    tol = 1e-7
    for kind in range(1, 8):
        ref = e.get_vars(kind)
        if len(ref):
            for k in range(world):
                assert rel(r[k][f"v{kind}"], ref) < tol, kind
    # one host read of the LM scalars per iteration that keeps its full step (the reduced scalars of
    # linearize, model reduction, step ratios and cost pass read together); the step-rescaling path
    # reads phase by phase, as Optimizer.cpp:907-1011 does
    reads = r[0]["reads"]
    assert len(reads) == s.num_iterations
    assert all(n == 1 for n, resc in reads if not resc), reads
    pts = np.where(r[0]["own"][:, None], r[0]["pts"], r[1]["pts"])
    assert np.all(r[0]["own"] ^ r[1]["own"] | ~(r[0]["own"] | r[1]["own"]))
    assert rel(pts, e.get_vars(0)) < tol


def _part_worker(rank, world, port, which, its, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    import torch.distributed as dist
    from oracle.refcpu import RefEngine
    from visual_inertial_bundle_adjustment_amd import synth
    from visual_inertial_bundle_adjustment_amd.distributed import PartitionedOptimizer, ShardComm

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = synth.generate(synth.config(which))
    e = RefEngine(imu_calib_options=p.imu_calib_options)
    e.set_partition(rank, world)
    synth.load_into(e, p)
    s = PartitionedOptimizer(e, ShardComm(rank, world, None)).optimize(_settings(its))
    res = {"iters": s.num_iterations, "initial": s.initial_cost, "final": s.final_cost}
    for k in range(1, 8):
        res[f"v{k}"] = e.get_vars(k)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_partitioned_controller_matches_single_process(world, tmp_path):
    """distributed.PartitionedOptimizer (the default multi-GPU mode) on gloo CPU ranks over the oracle's
    restatement of the partition protocol (refcpu.cpp ref_set_partition & co.: every exchange the HIP
    engine makes -- ROOT tiles and forward rows reduced to rank 0, ROOT factor + solve there, x rows
    broadcast, x shared by all-reduce, per-rank back-substitution of its landmarks -- carries the whole
    partial system here): same LM trajectory as the single-process oracle."""
    from oracle.refcpu import RefEngine
    from parity_util import make, rel
    which, its = "miniB", 6
    mp.spawn(_part_worker, args=(world, _free_port(), which, its, str(tmp_path)), nprocs=world, join=True)
    r = [dict(np.load(tmp_path / f"rank{k}.npz")) for k in range(world)]
    e, _ = make(RefEngine, which)
    s = e.optimize(_settings(its))
    for k in range(world):
        assert int(r[k]["iters"]) == s.num_iterations
        assert abs(float(r[k]["initial"]) - s.initial_cost) <= 1e-11 * s.initial_cost
        assert abs(float(r[k]["final"]) - s.final_cost) <= 1e-9 * s.final_cost
        for kind in range(1, 8):
            ref = e.get_vars(kind)
            if len(ref):
                assert rel(r[k][f"v{kind}"], ref) < 1e-7, kind


def _words_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    from visual_inertial_bundle_adjustment_amd.distributed import bits_word, word_bits

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank 0: RS lookup out of range (err[0] bit 0) and a preintegration gap (err[1] bit 3); rank 1: reduced
    # Cholesky breakdown (err[0] bit 3) and the cost pass's RS range (bit 5)
    words = [np.array([1, 8], np.int32), np.array([8 | 32, 0], np.int32)][rank]
    t = torch.tensor(word_bits(words), dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    np.save(os.path.join(out_dir, f"w{rank}.npy"), bits_word(t.tolist()))
    dist.destroy_process_group()


def test_error_words_ored_over_ranks(tmp_path):
    """The multi-process controllers combine the ranks' error bit words by a MAX over one 0/1 per bit, i.e. a
    bitwise OR (distributed.word_bits / bits_word): a MAX of the words themselves would keep only the
    larger (bit 8 over bit 1), and the causal-order decode (vb_error_from_words) would then report the
    reduced-system breakdown instead of the rolling-shutter range error a single process reports."""
    world = 2
    mp.spawn(_words_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert np.load(tmp_path / f"w{r}.npy").tolist() == [1 | 8 | 32, 8]
