"""potrf / trsm launch time for one tile (vb_bench_kernel), under the current VIBA_POTRF_WAVES / VIBA_DIAG_INV."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_inertial_bundle_adjustment_amd import synth  # noqa: E402
from visual_inertial_bundle_adjustment_amd.engine import HipEngine  # noqa: E402

p = synth.generate(synth.config("A"))
e = HipEngine(imu_calib_options=p.imu_calib_options)
synth.load_into(e, p)
tag = f"waves={os.environ.get('VIBA_POTRF_WAVES', '4')} inv={os.environ.get('VIBA_DIAG_INV', 'lds')}"
print(f"{tag}: potrf {e.bench_kernel(0, 200):.2f} us, trsm {e.bench_kernel(1, 200):.2f} us", flush=True)
