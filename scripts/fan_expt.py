"""Fan-in memory experiment: time every fan-in launch of one factorization (HIP events, family 4) with the
normal library and with a build whose fan-in reads the same few tiles for every contribution
(-DVIBA_FAN_EXPT, lib_expt/).  The second run's numbers are garbage; only its timing is used."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from visual_inertial_bundle_adjustment_amd import synth  # noqa: E402
from visual_inertial_bundle_adjustment_amd.engine import HipEngine  # noqa: E402

p = synth.generate(synth.config(sys.argv[1] if len(sys.argv) > 1 else "C"))
e = HipEngine(imu_calib_options=p.imu_calib_options)
synth.load_into(e, p, rs_device=True)
st = e.problem_stats()
out = []
for it in range(3):
    e.profile_kernel(4)
    e.linearize(True, False)
    try:
        e.damp_factor_solve(1e-5)
    except Exception as ex:  # the experiment build breaks the factor
        pass
    n, ms = e.kernel_time()
    e.profile_kernel(-1)
    out.append((n, ms))
flops = st[6] * 2.0 * 64 ** 3
print(json.dumps({"lib": os.environ.get("VIBA_LIB_DIR", "lib"), "launches_ms": out,
                  "tflops": [flops / (ms * 1e-3) / 1e12 for _, ms in out]}))
