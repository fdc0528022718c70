"""Phase cycles of schur_run2_kernel (library built with -DVIBA_SCHUR_TIMING into $VIBA_LIB_DIR): per-wave
s_memtime sums over one LM iteration on config C, as shares of the waves' total cycles."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_inertial_bundle_adjustment_amd import synth  # noqa: E402
from visual_inertial_bundle_adjustment_amd.engine import HipEngine, Settings  # noqa: E402

p = synth.generate(synth.config(sys.argv[1] if len(sys.argv) > 1 else "C"))
e = HipEngine(imu_calib_options=p.imu_calib_options)
synth.load_into(e, p)
st = Settings.default(max_num_iterations=1, stop_if_no_improvement_for=10**6, distance_from_troubled_iteration=0)
e.optimize(st)
t = (C.c_ulonglong * 8)()
e.lib.vb_debug_schur_times(t, 1)
e.optimize(st)
e.synchronize()
e.lib.vb_debug_schur_times(t, 0)
t = list(t)
names = ["setup (ecol, C clear)", "run scan", "tasks", "  k-loops + epilogues", "  rhs", "final barrier wait",
         "write-back"]
tot = t[0] + t[1] + t[2] + t[5] + t[6]
print(f"waves {t[7]}, cycles per wave {tot / max(1, t[7]):.0f}")
for i, n in enumerate(names):
    print(f"{n:26s} {t[i] / max(1, t[7]):10.0f} cycles/wave  {100.0 * t[i] / max(1, tot):5.1f} %")
