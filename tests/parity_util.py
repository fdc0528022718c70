"""Shared helpers for parity tests: run one LM step on two engines and compare."""
from __future__ import annotations

import numpy as np

from visual_inertial_bundle_adjustment_amd import synth
from visual_inertial_bundle_adjustment_amd.kinds import NUM_VAR_KINDS


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    den = max(np.abs(b).max(initial=0.0), 1e-300)
    return float(np.abs(a - b).max(initial=0.0) / den)


def one_step(engine, lam=1e-5):
    """linearize -> damp/factor/solve -> apply step -> comparable cost (Optimizer.cpp:807-897)."""
    out = {}
    out["cost0"] = engine.linearize(True, False)
    out["grad"] = [engine.get_gradient(k) for k in range(NUM_VAR_KINDS - 1)]
    out["model_red"] = engine.damp_factor_solve(lam)
    out["step"] = [engine.get_step(k) for k in range(NUM_VAR_KINDS - 1)]
    engine.backup()
    out["ratios"] = engine.apply_step(0)
    out["cost1"], out["stats1"] = engine.cost(True)
    out["vars1"] = [engine.get_vars(k) for k in range(NUM_VAR_KINDS - 1)]
    out["back_red"] = engine.gradient_dot_step(False)
    engine.solve_with_new_gradient()
    out["substep"] = [engine.get_step(k, 1) for k in range(NUM_VAR_KINDS - 1)]
    engine.restore()
    out["cost_restored"], _ = engine.cost(False)
    return out


def make(engine_cls, which="A", **kw):
    p = synth.generate(synth.config(which, **kw))
    e = engine_cls(imu_calib_options=p.imu_calib_options)
    synth.load_into(e, p)
    return e, p
