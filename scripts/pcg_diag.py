"""PCG GPU vs oracle divergence by iteration count (identity / Jacobi preconditioner, miniB)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from oracle.refcpu import RefEngine  # noqa: E402
from parity_util import make, rel  # noqa: E402
from visual_inertial_bundle_adjustment_amd.engine import HipEngine  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "miniB"
for solver in (1, 2):
    for lam in (1e-5, 1e-2):
        for its in (1, 2, 5, 10, 20, 40):
            out = []
            for cls in (HipEngine, RefEngine):
                e, _ = make(cls, which)
                e.set_solver(solver, its, 1e-30)
                e.linearize(True, False)
                m = e.damp_factor_solve(lam)
                out.append((m, [e.get_step(k) for k in range(8)], e.pcg_stats()))
            d = max(rel(out[0][1][k], out[1][1][k]) for k in range(8) if out[1][1][k].size)
            print(f"solver {solver} lam {lam:g} its {its:3d}: model_red rel {abs(out[0][0] - out[1][0]) / abs(out[1][0]):.2e} "
                  f"step rel {d:.2e} res gpu {out[0][2][1]:.3e} ref {out[1][2][1]:.3e}", flush=True)
