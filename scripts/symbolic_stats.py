"""Print the finalize-time diagnostics of the Schur work list and the tile Cholesky (VIBA_SCHUR_STATS,
VIBA_FACTOR_STATS) for one configuration: python scripts/symbolic_stats.py [C]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("VIBA_SCHUR_STATS", "1")
os.environ.setdefault("VIBA_FACTOR_STATS", "1")
from visual_inertial_bundle_adjustment_amd import synth  # noqa: E402
from visual_inertial_bundle_adjustment_amd.engine import HipEngine  # noqa: E402

p = synth.generate(synth.config(sys.argv[1] if len(sys.argv) > 1 else "C"))
e = HipEngine(imu_calib_options=p.imu_calib_options)
synth.load_into(e, p)
print(e.problem_stats(), flush=True)
e.close()
