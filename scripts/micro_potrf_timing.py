"""Phase timing of potrf_kernel (library built with -DVIBA_POTRF_TIMING into $VIBA_LIB_DIR)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_inertial_bundle_adjustment_amd import synth  # noqa: E402
from visual_inertial_bundle_adjustment_amd.engine import HipEngine  # noqa: E402

p = synth.generate(synth.config("A"))
e = HipEngine(imu_calib_options=p.imu_calib_options)
synth.load_into(e, p)
print("potrf us", e.bench_kernel(0, 50))
t = (C.c_longlong * 32)()
e.lib.vb_debug_potrf_times(t)
t = list(t)
base = t[19]
names = {19: "start", 16: "loaded"}
for i in range(4):
    names[4 * i] = f"row{i} begin"
    names[4 * i + 1] = f"row{i} trsm done"
    names[4 * i + 2] = f"row{i} S done"
    names[4 * i + 3] = f"row{i} diag16 done"
names[17] = "factored"
names[18] = "stored"
for k in [19, 16] + list(range(16)) + [17, 18]:
    print(f"{names[k]:20s} {t[k] - base:8d} cycles")
