"""Per-kernel times of the linearize / Schur phases on config C, each kernel alone (vb_bench_kernel 10-15),
after two LM iterations from the generator's x0, for both precision builds.

    python scripts/kernel_probe.py [config=C] [iters=5] [precisions=fp64,mixed] [kernels=10,11,...]
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_inertial_bundle_adjustment_amd import synth  # noqa: E402
from visual_inertial_bundle_adjustment_amd.engine import HipEngine, Settings  # noqa: E402

NAMES = {0: "potrf4 (one tile, scratch)", 1: "trsm (one tile, scratch)", 2: "fan-in (one pair, scratch)",
         10: "visual_lin (eval + record stores)", 12: "landmark elimination",
         13: "observation-group Gram blocks", 14: "Schur tile products", 15: "visual cost pass",
         16: "small factors' evaluation", 17: "small assembly, IMU kinds", 18: "small assembly, other kinds",
         19: "reduced-system clear", 20: "elimination beside tile products (timing probe)",
         21: "elimination then tile products", 22: "elimination beside groups",
         23: "factorization (its streams)", 24: "factorization beside tile products (timing probe)",
         25: "factorization beside tile products on stZ (timing probe)"}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    precs = sys.argv[3].split(",") if len(sys.argv) > 3 else ["fp64", "mixed"]
    which = [int(w) for w in sys.argv[4].split(",")] if len(sys.argv) > 4 else list(NAMES)
    p = synth.generate(synth.config(cfg))
    out = {}
    for prec in precs:
        e = HipEngine(imu_calib_options=p.imu_calib_options, precision=prec)
        synth.load_into(e, p, rs_device=True)
        try:  # records and staging in place (a diagnostic build may not converge)
            e.optimize(Settings.default(max_num_iterations=2, stop_if_no_improvement_for=10**6,
                                        distance_from_troubled_iteration=0))
        except Exception as ex:
            print(f"[probe] optimize: {ex}", file=sys.stderr)
        f = e._fn("bench_kernel", [C.c_int, C.c_int, C.POINTER(C.c_double)])
        res = {}
        for w in which:
            us = C.c_double()
            e._check(f(e.h, w, iters, C.byref(us)))
            res[NAMES[w]] = round(us.value, 1)
        out[prec] = res
        e.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
