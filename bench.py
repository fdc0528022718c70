#!/usr/bin/env python
"""LM iterations/s of the MI355X VI-BA engine on the synthetic config-C problem.

Metric (BASELINE.json): "LM iterations/sec (and ms/iter) on 10k-pose/300k-landmark VI-BA".
One step = one iteration of Optimizer::optimize (Optimizer.cpp:800-1097) as ark_vi_ba drives it: the
preStepCallback's rolling-shutter table rebuild from the IMU stream (main_AriaKit_ViBa.cpp:95-101), linearize all factors,
damp + Schur-eliminate landmarks + factor + solve the reduced system, box-plus, cost pass, and the
LM accept/reject (+ rescaled / sub-step attempts when the step is bad), as driven by vb_optimize.

    python bench.py [--gpus N --steps K --warmup W --config C]

N > 1 runs under torch.distributed (one rank per GPU): landmarks are sharded in time-banded
ranges, every rank linearizes/eliminates its shard, the partial reduced systems are summed on
rank 0 over RCCL, rank 0 factors/solves and broadcasts the reduced step.
Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# kernel families of vb_profile_kernel
KF_VISUAL_LIN, KF_LANDMARK, KF_SCHUR, KF_POTRF, KF_GEMM, KF_FWD, KF_BWD, KF_BACKSUB, KF_COST, KF_SMALL, KF_TRSM, \
    KF_SYMV = range(12)
SOLVERS = {"direct": 0, "pcg-trivial": 1, "pcg-jacobi": 2, "pcg-gauss-seidel": 3, "pcg-lower-prec": 4}
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
FP64_MFMA_PEAK_TF = 78.6   # MI355X fp64 matrix peak (spec)
# what the fp64 MFMA sustains on this chip with independent accumulators and no memory traffic
# (scripts/micro/mfma_peak.hip, profiles/r03_mfma_peak.txt): v_mfma_f64_4x4x4_4b 74.9 TF/s (NACC 8, 4
# workgroups per CU), the hardware's practical fp64 matrix ceiling; the 16x16x4 form the fan-in issues
# sustains 47.7 TF/s, a limit of that instruction, not of the chip
FP64_MFMA_4X4X4_MEASURED_TF = 74.9


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def visual_bytes_per_launch(p, nobs: int) -> float:
    """Algorithmic HBM bytes of one visual linearize launch: per observation
    48 B of constants, 6 int32 indices, the cached cost (read+write), the point (24 B) and the 72-plane
    whitened Jacobian record written (576 B); shared variables (poses, velocities, calibration) once."""
    per_obs = 48 + 6 * 4 + 16 + 24 + 72 * 8
    shared = sum(p.vars[k].nbytes for k in (1, 2, 4, 5))
    return nobs * per_obs + shared


def pmc_traffic(kernel: str, path: str | None = None):
    """(HBM bytes per launch of `kernel`, provenance) from the committed rocprofv3 PMC summary
    (profiles/pmc_summary.json, written by scripts/pmc_summary.py from separate FETCH_SIZE / WRITE_SIZE
    passes, FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM).  The bytes are None unless the summary was
    measured on exactly the HIP sources this tree builds (sources digest, build.sources_digest): a summary of
    other code is reported as stale, never as this binary's traffic."""
    from visual_inertial_bundle_adjustment_amd.build import sources_digest
    path = path or os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            summ = json.load(f)
    except (OSError, ValueError):
        return None, {"status": "missing"}
    meta = summ.get("_meta", {})
    here = sources_digest()
    prov = {"measured_at_commit": meta.get("commit"), "sources_sha256": meta.get("sources_sha256"),
            "tree_sources_sha256": here}
    if meta.get("sources_sha256") != here:
        prov["status"] = "stale: measured on other HIP sources than this tree's"
        return None, prov
    prov["status"] = "measured on this tree's HIP sources"
    try:
        return summ[kernel]["hbm_bytes_per_launch"], prov
    except KeyError:
        prov["status"] = f"no {kernel} entry"
        return None, prov


def host_threads() -> tuple[int, int]:
    """(threads for the 'nproc' baseline run, nproc).  On the GPU box os.cpu_count() reports the whole
    machine while the job's CPU share is OMP_NUM_THREADS (16), so the run uses the smaller of the two."""
    nproc = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", nproc) or nproc)
    return max(1, min(nproc, share)), nproc


def cpu_baseline(p, name: str = "C", repeats: int = 3, recompute_preint: bool = False, warmup: int = 0):
    """The CPU baseline of BASELINE.md, measured on the FULL workload (no slice, no extrapolation):
    oracle/refcpu (this repository's restatement of the reference path: factor functors, the LM loop,
    point elimination + blocked Cholesky) runs `warmup` untimed iterations (as the GPU bench does, so the
    timed iterations start from the same kind of state as the GPU's), then `repeats` individually timed
    full iterations of Optimizer::optimize at the job's thread count (value = 1 / median, with the
    spread), and one more at 8 threads (the reference's numThreads default, Optimizer.h:42 /
    Settings.h:87) for comparison.  Reports the median iteration's phase split."""
    import statistics

    from oracle.refcpu import RefEngine
    from visual_inertial_bundle_adjustment_amd import synth
    from visual_inertial_bundle_adjustment_amd.engine import Settings
    t = time.perf_counter()
    e = RefEngine(imu_calib_options=p.imu_calib_options)
    synth.load_into(e, p, rs_device=True, recompute_preint=recompute_preint)
    log(f"[bench] cpu baseline: oracle loaded in {time.perf_counter() - t:.1f}s")
    nthr, nproc = host_threads()

    def one_iteration():
        s = Settings.default(max_num_iterations=1, stop_if_no_improvement_for=10**6, distance_from_troubled_iteration=0)
        t0 = time.perf_counter()
        out = e.optimize(s)
        return (time.perf_counter() - t0) * 1e3 / max(1, out.num_iterations), e.phase_times()

    e.set_threads(nthr)
    if warmup:
        t = time.perf_counter()
        e.optimize(Settings.default(max_num_iterations=warmup, stop_if_no_improvement_for=10**6,
                                    distance_from_troubled_iteration=0))
        log(f"[bench] cpu baseline: {warmup} warmup iteration(s) in {time.perf_counter() - t:.1f}s")
    e.backup()
    runs = [one_iteration() for _ in range(repeats)]
    ms = [r[0] for r in runs]
    med = statistics.median(ms)
    ph = runs[ms.index(sorted(ms)[len(ms) // 2])][1]
    log(f"[bench] cpu baseline {nthr} threads: iterations {', '.join(f'{x:.0f}' for x in ms)} ms (median {med:.0f})")
    out8 = None
    if nthr != 8:  # the reference's default thread count, one iteration from the same state as the first
        e.restore()
        e.set_threads(8)
        m8, ph8 = one_iteration()
        out8 = {"ms_per_step": m8, "phases_ms": {k: round(v, 1) for k, v in ph8.items()}}
        log(f"[bench] cpu baseline 8 threads: {m8:.0f} ms/iteration")
    return {"value": 1e3 / med, "unit": "LM iterations/s", "cores": nthr, "kind": "port", "nproc": nproc,
            "iterations_ms": [round(x, 1) for x in ms], "median_ms": med, "min_ms": min(ms), "max_ms": max(ms),
            "spread": (max(ms) - min(ms)) / med, "phases_ms": {k: round(v, 1) for k, v in ph.items()},
            "threads_8": out8,
            "sample": f"{repeats} individually timed full LM iterations of oracle/refcpu on the whole config-{name} "
                      f"problem ({p.num_obs} obs) at {nthr} threads (nproc {nproc}) after {warmup} untimed warmup "
                      f"iteration(s); value = 1 / median; one more iteration at 8 threads for comparison"}


def mixed_vs_fp64(p, device, rs_device):
    """Config E tolerance: one LM step (linearize, damp + factor + solve) from the same x0 on
    the fp64 and the mixed-precision engines; ||delta_E - delta_C|| / ||delta_C|| over all variables, the
    model cost reductions, and the costs after applying each step."""
    import numpy as np
    from visual_inertial_bundle_adjustment_amd import synth
    from visual_inertial_bundle_adjustment_amd.engine import HipEngine
    out = {}
    for prec in ("fp64", "mixed"):
        e = HipEngine(imu_calib_options=p.imu_calib_options, device=device, precision=prec)
        synth.load_into(e, p, rs_device=rs_device)
        c0 = e.linearize(True, False)
        mr = e.damp_factor_solve(1e-5)
        step = np.concatenate([e.get_step(k).ravel() for k in range(8)])
        e.backup()
        e.apply_step(0)
        c1, _ = e.cost(True)
        out[prec] = (c0, mr, step, c1)
        e.close()
    (c0, mr, s64, c164), (_, mrm, smx, c1mx) = out["fp64"], out["mixed"]
    return {"step_rel_l2": float(np.linalg.norm(smx - s64) / np.linalg.norm(s64)),
            "step_rel_max": float(np.abs(smx - s64).max() / np.abs(s64).max()),
            "model_reduction_rel": float(abs(mrm - mr) / abs(mr)),
            "cost_after_step": {"fp64": c164, "mixed": c1mx}, "cost_before": c0}


def banded_contributions(p, device, rs_device, precision):
    """Tile-pair contributions of the reduced system's Cholesky in the time order (a nested-dissection
    leaf larger than the whole system: one part, in time order), from a second handle that is only
    finalized."""
    from visual_inertial_bundle_adjustment_amd import synth
    from visual_inertial_bundle_adjustment_amd.engine import HipEngine
    prev = os.environ.get("VIBA_ND_LEAF")
    os.environ["VIBA_ND_LEAF"] = str(1 << 62)
    try:
        eb = HipEngine(imu_calib_options=p.imu_calib_options, device=device, precision=precision)
        try:
            synth.load_into(eb, p, rs_device=rs_device)
            return int(eb.problem_stats()[6])
        finally:
            eb.close()
    finally:
        if prev is None:
            del os.environ["VIBA_ND_LEAF"]
        else:
            os.environ["VIBA_ND_LEAF"] = prev


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: run this script under torch.distributed.run with N ranks
    (one per GPU, RCCL) as a child process, before anything here touches a GPU, and return its exit code
    (the driver's own N > 1 form sets WORLD_SIZE and never comes here)."""
    import subprocess
    # a standalone c10d rendezvous: its store binds a free port itself (no probe-then-bind port race), and
    # the workers reach it at 127.0.0.1 (the container hostname may not resolve)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--standalone",
           "--local-addr", "127.0.0.1", os.path.abspath(__file__), *sys.argv[1:]]
    log(f"[bench] launching {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU).  Under torch.distributed.run it must equal WORLD_SIZE; without it, "
                         "N > 1 launches torch.distributed.run with N ranks as a child process")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-family", type=int, default=KF_GEMM,
                    help="kernel family whose launches a separate pass after the timed one event-times for the "
                         "roofline (-1: none)")
    ap.add_argument("--profile-steps", type=int, default=3, help="LM iterations of the profiled pass")
    ap.add_argument("--precision", choices=("fp64", "mixed"), default="fp64",
                    help="fp64 (the reference's arithmetic) or mixed (config E: fp32 Jacobian records and "
                         "Schur-complement products, fp64 Cholesky); mixed also reports its first-step "
                         "deviation from fp64")
    ap.add_argument("--refine", action="store_true",
                    help="run refinePoints before the LM loop, as ark_vi_ba (untimed; it changes the LM trajectory, "
                         "so the default times the loop from the generator's x0 like earlier rounds)")
    ap.add_argument("--rs-tables", choices=("device", "host"), default="device",
                    help="device: rebuild the rolling-shutter tables from the IMU stream at the start of every "
                         "iteration (ark_vi_ba's preStepCallback); host: fixed precomputed tables")
    ap.add_argument("--solver", choices=tuple(SOLVERS), default="direct",
                    help="reduced-system solver (Optimizer::Settings solverType): the tile Cholesky, or PCG with "
                         "the identity / block-Jacobi / block-Gauss-Seidel / fp32-Cholesky preconditioner")
    ap.add_argument("--pcg-iterations", type=int, default=40, help="pcgMaxIterations (Optimizer.h:44)")
    ap.add_argument("--pcg-residual", type=float, default=1e-10, help="pcgDesiredResidual (Optimizer.h:45)")
    ap.add_argument("--no-banded-count", action="store_true",
                    help="skip the symbolic analysis of the time-ordered (banded) reduced system that prices the "
                         "factorization against the banded flop count")
    ap.add_argument("--recompute-preint", action="store_true",
                    help="ark_vi_ba --recompute-preint: every iteration re-preintegrates every inertial factor "
                         "from the IMU stream on the device (preint.hip)")
    args = ap.parse_args()
    if args.solver != "direct" and args.profile_family == KF_GEMM:
        args.profile_family = KF_SYMV  # no fan-in without the factorization: the PCG product instead

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        return spawn_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world:
        log(f"[bench] --gpus {args.gpus} but WORLD_SIZE {world}: one rank per GPU is expected")
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        from visual_inertial_bundle_adjustment_amd.distributed import run_sharded
        return run_sharded(args, rank, world, local)

    from visual_inertial_bundle_adjustment_amd import synth
    from visual_inertial_bundle_adjustment_amd.engine import HipEngine, Settings

    t = time.perf_counter()
    p = synth.generate(synth.config(args.config))
    log(f"[bench] config {args.config}: {p.summary()} (generated in {time.perf_counter() - t:.1f}s)")
    t = time.perf_counter()
    tolerance = None
    if args.precision == "mixed":
        tolerance = mixed_vs_fp64(p, local, args.rs_tables == "device")
        log(f"[bench] mixed vs fp64, first LM step: {tolerance}")
    e = HipEngine(imu_calib_options=p.imu_calib_options, device=local, precision=args.precision)
    synth.load_into(e, p, rs_device=args.rs_tables == "device", recompute_preint=args.recompute_preint)
    e.set_solver(SOLVERS[args.solver], args.pcg_iterations, args.pcg_residual)
    st = e.problem_stats()
    sched = e.factor_schedule_stats()
    log(f"[bench] factorization schedule: {sched[0]} levels, {sched[1]} fan-in contributions, {sched[3]} of "
        f"{sched[2]} supernodes two-column")
    log(f"[bench] finalize {time.perf_counter() - t:.1f}s; reduced order {st[3]}, tiles {st[5]} "
        f"({st[4]} tile columns, {st[10]} levels), gemm pairs/factorization {st[6]}, Schur entries: landmark-tile {st[8]}, obs-pair {st[9]}")

    # ark_vi_ba's order (main_AriaKit_ViBa.cpp:66-102): rolling-shutter tables (done at load), point
    # refinement, then the LM loop; the refinement is a one-off before the loop and is not timed
    if args.refine:
        e.synchronize()
        t = time.perf_counter()
        (c0, c1), (nf, nit, nmov) = e.refine_points()
        e.synchronize()
        log(f"[bench] refinePoints {1e3 * (time.perf_counter() - t):.1f} ms: visual cost {c0:.6g} -> {c1:.6g}, "
            f"{nit} iterations, {nmov} points moved, {nf} failures")

    # run exactly W then K iterations of the optimize loop (convergence stops disabled)
    def settings(n):
        return Settings.default(max_num_iterations=n, stop_if_no_improvement_for=10**6,
                                distance_from_troubled_iteration=0)
    if args.warmup:
        s = e.optimize(settings(args.warmup))
        log(f"[bench] warmup {s.num_iterations} its, cost {s.initial_cost:.6g} -> {s.final_cost:.6g}")
    e.synchronize()
    t0 = time.perf_counter()
    s = e.optimize(settings(args.steps))
    e.synchronize()
    elapsed = time.perf_counter() - t0
    iters = s.num_iterations
    ph = e.phase_times()
    log(f"[bench] timed {iters} its in {elapsed:.3f}s, cost {s.initial_cost:.6g} -> {s.final_cost:.6g}; "
        f"last it: lin {ph.linearize_ms:.2f} schur {ph.schur_ms:.2f} factor {ph.factor_ms:.2f} "
        f"solve {ph.solve_ms:.2f} step {ph.step_ms:.2f} cost {ph.cost_ms:.2f} rs-tables {ph.rs_update_ms:.3f} ms")
    # the roofline's kernel timing: a separate pass of the same binary with the profiled family's launches
    # event-timed one by one, on the same multi-stream schedule as the timed pass: a launch can share the
    # chip with the other stream's, so the roofline divides by the family's busy time (the union of its
    # launch intervals, vb_kernel_busy_time), not by the sum of launch durations
    prof_iters = 0
    launches, kms, busy_ms = 0, 0.0, 0.0
    if args.profile_family >= 0 and args.profile_steps > 0:
        e.profile_kernel(args.profile_family)
        sp = e.optimize(settings(args.profile_steps))
        e.synchronize()
        launches, kms = e.kernel_time()
        busy_ms = e.kernel_busy_time()
        e.profile_kernel(-1)
        prof_iters = sp.num_iterations
        log(f"[bench] profiled pass: {prof_iters} its, {launches} launches of family {args.profile_family}, "
            f"{kms:.3f} ms")

    # roofline of the profiled kernel family (average launch duration from HIP events on the engine
    # stream, algorithmic work from the symbolic structure)
    avg_ms = kms / max(1, launches)
    if args.profile_family < 0 or launches == 0 or kms <= 0:
        # nothing event-timed (the factorization ran from its HIP graph, or the family never launched)
        roof = None
    elif args.profile_family == KF_GEMM:
        # st[6] tile-pair contributions per factorization (2 * 64^3 flops each); one factorization per
        # LM iteration (the rescaled / sub-step attempts reuse it), and the launches are the fan-in
        # launches actually timed (levels without contributions launch none: 88 of the 89 levels at
        # config C), so flops per launch = contributions x iterations / launches
        fan_per_factor = launches / max(1, prof_iters)
        # the fan-in's own contributions (the two-column supernode schedule moves the pair-internal ones
        # into its trsm kernel; the column schedule's are st[6])
        fan_contrib = sched[1]
        per_launch = fan_contrib * 2.0 * 64 ** 3 / max(1e-9, fan_per_factor)
        # the factorization's streams run fan-in launches side by side, so a launch's own duration counts
        # time it shares with another: the duration per launch is the family's busy time (the union of
        # its launches' intervals) over the launches -- the plain average when nothing overlaps
        eff_ms = busy_ms / max(1, launches)
        achieved = per_launch / (eff_ms * 1e-3) / 1e12
        # compulsory HBM bytes of one launch: within a level every contribution's L_IK is a distinct
        # tile (a column K has at most one ancestor column per level) and every L_JK is also the
        # I-side tile of the diagonal contribution (J, J, K), so the operands are pairs x 32 KB; each
        # target tile is read and written once (st[5] tiles over the launches bounds the targets)
        compulsory = (fan_contrib * 64 * 64 * 8 + st[5] * 2 * 64 * 64 * 8) / max(1e-9, fan_per_factor)
        traffic, tprov = pmc_traffic("fanin_kernel")
        roof = {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TF, "unit": "TFLOP/s",
                "frac": achieved / FP64_MFMA_PEAK_TF, "traffic": traffic, "traffic_provenance": tprov,
                "compulsory_bytes_per_launch": compulsory,
                "traffic_over_compulsory": traffic / compulsory if traffic else None,
                "kernel": "fanin_kernel (level-batched fan-in tile update A_IJ -= sum_K L_IK L_JK^T on "
                          "v_mfma_f64_16x16x4_f64, operands via global_load_lds)",
                "flops_per_launch": per_launch, "busy_ms_per_launch": eff_ms, "avg_launch_ms": avg_ms,
                "launches": launches, "busy_ms_per_factorization": busy_ms / max(1, prof_iters),
                "frac_per_launch_duration": per_launch / (avg_ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TF,
                "fanin_launches_per_factorization": fan_per_factor, "levels": int(sched[0]),
                "fanin_contributions": int(fan_contrib), "supernodes": int(sched[2]),
                "two_column_supernodes": int(sched[3]),
                "ceiling_4x4x4_measured": FP64_MFMA_4X4X4_MEASURED_TF,
                "frac_of_4x4x4_ceiling": achieved / FP64_MFMA_4X4X4_MEASURED_TF}
    elif args.profile_family == KF_SYMV:
        # every tile of S (stored tiles less the symbolic fill) once (32 KB) + x and y rows (1 KB) per launch
        b = st[11] * (64 * 64 * 8 + 2 * 64 * 8)
        achieved = b / (avg_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic("tile_symv_kernel")[0],
                "kernel": "tile_symv_kernel (PCG product y += S x over the lower tiles of S, fill skipped)",
                "bytes_per_launch": b, "avg_launch_ms": avg_ms, "launches": launches}
    else:
        b = visual_bytes_per_launch(p, st[0])
        achieved = b / (avg_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic("visual_lin_kernel")[0],
                "kernel": "visual_lin_kernel (Jacobian fill)", "bytes_per_launch": b, "avg_launch_ms": avg_ms,
                "launches": launches}
    if roof is not None:
        roof["timing"] = (f"HIP events around each launch on its own stream, in a separate pass of {prof_iters} LM "
                          f"iterations after the timed ones ({launches} launches)")
        if args.profile_family == KF_GEMM:
            roof["divisor"] = ("busy time: the factorization runs its independent subtrees on two streams, so fan-in "
                               "launches overlap and a launch's own duration (avg_launch_ms) includes time shared with "
                               "the other stream's launch; achieved = flops per factorization / the union of the "
                               "launches' intervals per factorization (busy_ms_per_launch = that union / launches, "
                               "the plain average when nothing overlaps); frac_per_launch_duration divides by "
                               "avg_launch_ms instead")
    ms = elapsed * 1e3 / max(1, iters)
    if tolerance is not None:
        out_extra = {"precision": "mixed (fp32 Jacobian records + Schur products, fp64 Cholesky)",
                     "vs_fp64": tolerance}
    else:
        out_extra = {}
    if args.solver != "direct":
        it, res = e.pcg_stats()
        out_extra["solver"] = {"type": args.solver, "max_iterations": args.pcg_iterations,
                               "desired_residual": args.pcg_residual, "last_iterations": it,
                               "last_relative_residual": res}
        log(f"[bench] last PCG solve: {it} iterations, relative residual {res:.3g}")
    out_extra["phases_ms"] = {k: round(getattr(ph, k), 3) for k, _ in ph._fields_}
    e.close()  # free the device before the banded analysis and the host run
    if roof is not None and args.profile_family == KF_GEMM and not args.no_banded_count:
        # the factorization against two flop counts: the nested-dissection order's (what runs) and the
        # time order's (the band the reference's supernodal solver would see without our reordering)
        t = time.perf_counter()
        try:
            banded = banded_contributions(p, local, args.rs_tables == "device", args.precision)
            nd_gf, band_gf = st[6] * 2.0 * 64 ** 3 / 1e9, banded * 2.0 * 64 ** 3 / 1e9
            roof["factor"] = {"factor_ms": ph.factor_ms, "contributions_nd": int(st[6]),
                              "contributions_banded": int(banded), "gflop_nd": nd_gf, "gflop_banded": band_gf,
                              "tflops_nd": nd_gf / ph.factor_ms, "tflops_banded": band_gf / ph.factor_ms,
                              "frac_nd": nd_gf / ph.factor_ms / FP64_MFMA_PEAK_TF,
                              "frac_banded": band_gf / ph.factor_ms / FP64_MFMA_PEAK_TF}
            log(f"[bench] banded analysis {time.perf_counter() - t:.1f}s: {banded} contributions "
                f"(nested dissection {st[6]})")
        except Exception as ex:
            log(f"[bench] banded analysis failed: {ex}")
    cpu = None
    if not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(p, args.config, recompute_preint=args.recompute_preint, warmup=args.warmup)
        except Exception as ex:  # the baseline must never hide the GPU number
            log(f"[bench] cpu baseline failed: {ex}")
    out = {"metric": "LM iterations/sec on 10k-pose/300k-landmark VI-BA", "value": iters / elapsed,
           "unit": "LM iterations/s", "n_gpus": 1, "steps": iters, "warmup": args.warmup,
           "ms_per_step": ms, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
           "dtype": "f64" if args.precision == "fp64" else "f32/f64",
           "data": "synthetic (seeded Aria-like generator, csrc/synth.cpp)",
           "config": {"workload": f"config {args.config}: {st[0]} obs, {st[1]} landmarks, "
                                  f"{p.vars[1].shape[0]} rigs, reduced order {st[3]}",
                      "rigs": int(p.vars[1].shape[0]), "landmarks": int(st[1]), "observations": int(st[0]),
                      "parallelism": "single GPU"},
           "roofline": roof, "cpu_baseline": cpu, **out_extra}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    sys.exit(main() or 0)
