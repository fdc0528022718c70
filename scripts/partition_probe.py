"""Per-rank work of the partitioned factorization (config C by default) on ONE GPU, ranks built one
after another: landmarks, subtree / ROOT columns, fan-in contributions, ROOT exchange volume, and
the device time of each rank's phases (linearize, Schur assembly, subtree factor, subtree solves;
rank 0 also the ROOT factor + solve, timed on its partial -- not summed -- ROOT tiles, so a numeric
breakdown there is expected and ignored).  Estimate of one LM iteration at N ranks:
max_r(lin + assemble + factor0 + fwd0) + exchange + root + max_r(bwd0) + back-substitution."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_inertial_bundle_adjustment_amd import synth  # noqa: E402
from visual_inertial_bundle_adjustment_amd.engine import HipEngine, VbError  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
worlds = [int(w) for w in (sys.argv[2] if len(sys.argv) > 2 else "1,2,8").split(",")]
reps = 3
p = synth.generate(synth.config(cfg))


def timed(e, fn, *a):
    best = 1e30
    for _ in range(reps):
        e.synchronize()
        t0 = time.perf_counter()
        try:
            fn(*a)
        except VbError:
            pass
        e.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


for world in worlds:
    for rank in range(world):
        t0 = time.perf_counter()
        e = HipEngine(imu_calib_options=p.imu_calib_options)
        if world > 1:
            e.set_partition(rank, world)
        synth.load_into(e, p)
        build = time.perf_counter() - t0
        info = e.part_info()
        st = e.problem_stats()
        lin = timed(e, e.linearize, True, False)

        def fresh():
            e.linearize(True, False)
            e.assemble_reduced(1e-4)

        asm = timed(e, fresh) - lin
        f0 = timed(e, lambda: (fresh(), e.synchronize(), e.factor_part(0))) - asm - lin
        s0 = timed(e, e.solve_part, 0)
        s2 = timed(e, e.solve_part, 2)
        root = 0.0
        if world > 1 and rank == 0:
            root = timed(e, e.solve_part, 1)
            root += timed(e, lambda: (fresh(), e.factor_part(0), e.synchronize(), e.factor_part(1))) - asm - lin - f0
        bs = timed(e, e.back_substitute, 0)
        print(f"W={world} r={rank}: build {build:.1f}s  cols own {info[0]} root {info[1]}  pairs local {info[2]} "
              f"root {info[3]}  root tiles {info[4]} ({info[4] * 32768 / 1e6:.0f} MB)  Schur lm-entries {st[8]}  | "
              f"lin {lin:.2f} asm {asm:.2f} factor0 {f0:.2f} fwd0 {s0:.2f} bwd0 {s2:.2f} root {root:.2f} "
              f"backsub {bs:.2f} ms", flush=True)
        e.close()
