import sys, time, numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "./tests")
from visual_inertial_bundle_adjustment_amd.engine import HipEngine
from oracle.refcpu import RefEngine
from parity_util import one_step, make, rel
from visual_inertial_bundle_adjustment_amd.kinds import VAR_NAMES
for which in ["A", "miniB"]:
    g, p = make(HipEngine, which)
    r, _ = make(RefEngine, which)
    print(which, p.summary(), "red order", g.reduced_order(), r.reduced_order(), flush=True)
    t = time.time(); og = one_step(g); tg = time.time() - t
    t = time.time(); orf = one_step(r); tr = time.time() - t
    print(f"  gpu {tg:.3f}s cpu {tr:.3f}s")
    for k in ["cost0", "model_red", "cost1", "back_red", "cost_restored"]:
        print(f"  {k}: gpu {og[k]!r} ref {orf[k]!r} rel {abs(og[k]-orf[k])/max(abs(orf[k]),1e-300):.3e}")
    print("  stats", og["stats1"], orf["stats1"], "ratios", og["ratios"], orf["ratios"])
    for k in range(8):
        if len(og["step"][k]):
            print(f"  {VAR_NAMES[k]:10s} grad {rel(og['grad'][k], orf['grad'][k]):.2e} step {rel(og['step'][k], orf['step'][k]):.2e} sub {rel(og['substep'][k], orf['substep'][k]):.2e} vars {rel(og['vars1'][k], orf['vars1'][k]):.2e}")
    sg = g.optimize(); sr = r.optimize()
    print("  optimize gpu", sg.initial_cost, sg.final_cost, sg.num_iterations, " ref", sr.initial_cost, sr.final_cost, sr.num_iterations, flush=True)
