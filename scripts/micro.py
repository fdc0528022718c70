"""Micro-benchmark of the factorization kernels (vb_bench_kernel) on scratch tiles."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_inertial_bundle_adjustment_amd import synth  # noqa: E402
from visual_inertial_bundle_adjustment_amd.engine import HipEngine  # noqa: E402

p = synth.generate(synth.config("A"))
e = HipEngine(imu_calib_options=p.imu_calib_options)
synth.load_into(e, p)
for which, name in enumerate(["potrf", "trsm", "update+potrf", "update"]):
    print(f"{name:14s} {e.bench_kernel(which, 300):8.2f} us", flush=True)
