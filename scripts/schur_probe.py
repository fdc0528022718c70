"""Average duration of the Schur pass (KF_SCHUR: damping, observation groups, the tile-product kernel) on
config C with HIP events, independent of the values it produces (for the diagnostic VIBA_SCHUR_EXPT builds,
whose S is garbage: the factorization's breakdown is caught)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_inertial_bundle_adjustment_amd import synth  # noqa: E402
from visual_inertial_bundle_adjustment_amd.engine import HipEngine, VbError  # noqa: E402

p = synth.generate(synth.config(sys.argv[1] if len(sys.argv) > 1 else "C"))
e = HipEngine(imu_calib_options=p.imu_calib_options)
synth.load_into(e, p)
for k in range(6):
    if k == 1:
        e.profile_kernel(2)  # KF_SCHUR
    e.linearize(True, False)
    try:
        e.damp_factor_solve(1e-4)
    except VbError:
        pass
e.synchronize()
n, ms = e.kernel_time()
print(f"{os.environ.get('VIBA_LIB_DIR', 'lib').split('/')[-1]} {os.environ.get('VIBA_SCHUR_V', '')}: Schur pass "
      f"{ms / max(1, n):.3f} ms ({n} launches)")
