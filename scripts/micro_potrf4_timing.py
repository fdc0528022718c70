"""Phase timing of potrf4_kernel (library built with -DVIBA_POTRF_TIMING into $VIBA_LIB_DIR): cycle stamps
of wave 0 (start, end of the loop, stored), wave k around its diag16, wave 3 after each step's barrier."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_inertial_bundle_adjustment_amd import synth  # noqa: E402
from visual_inertial_bundle_adjustment_amd.engine import HipEngine  # noqa: E402

p = synth.generate(synth.config("A"))
e = HipEngine(imu_calib_options=p.imu_calib_options)
synth.load_into(e, p)
print(os.environ.get("VIBA_DIAG_INV", "dpp"), "potrf us", e.bench_kernel(0, 50))
t = (C.c_longlong * 32)()
e.lib.vb_debug_potrf_times(t)
t = list(t)
names = {0: "start"}
for k in range(4):
    names[1 + 2 * k] = f"diag16({k}) begin"
    names[2 + 2 * k] = f"diag16({k}) end"
    names[9 + k] = f"w3 after B1({k})"
    names[15 + 3 * k] = f"  chol16({k}) begin"
    names[16 + 3 * k] = f"  chol16({k}) end"
    names[17 + 3 * k] = f"  inv16({k}) end"
names[13] = "loop done"
names[14] = "stored"
for k in sorted([k for k in names if t[k]], key=lambda k: t[k]):
    print(f"{names[k]:20s} {t[k] - t[0]:8d} cycles")
