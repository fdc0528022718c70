"""Covariances (Optimizer::computeCovariances / computeJointCovariances,
lib/small_thing/Optimizer.cpp:503-697).  The reference's own check, TestOptimizer.cpp:50-83 (block
covariances of the spring chain equal the diagonal of the inverse damped Hessian to 1e-7; the joint
covariance of {1, 3, 4} times their marginal information matrix is the identity to 1e-9), is restated on
the oracle (CPU) and on the HIP engine (GPU, through the C-ABI vb_compute_covariances), and the GPU is
compared with the oracle on the synthetic VI-BA problems."""
from __future__ import annotations

import numpy as np
import pytest

from parity_util import make, make_spring_chain
from visual_inertial_bundle_adjustment_amd.engine import Settings
from visual_inertial_bundle_adjustment_amd.kinds import VAR_CAM_INTR

DAMPING = Settings.default().damping  # computeCovariances({}) uses the default Settings (damping 1e-5)


def _spring_hessian(n=6, lam=DAMPING):
    """the damped Hessian of the chain's first parameter (addDamping: d (1 + lambda) + lambda)"""
    D = np.zeros((n - 1, n))
    for i in range(n - 1):
        D[i, i], D[i, i + 1] = -1.0, 1.0
    H = D.T @ D
    H[np.diag_indices(n)] = H[np.diag_indices(n)] * (1 + lam) + lam
    return H


def _kat(engine_cls):
    e = make_spring_chain(engine_cls)
    e.optimize(Settings.default())
    covs, used = e.compute_covariances([[(VAR_CAM_INTR, i)] for i in range(6)], DAMPING)
    assert used == DAMPING
    H = _spring_hessian()
    inv = np.linalg.inv(H)
    for i, c in enumerate(covs):
        assert c.shape == (4, 4)
        assert abs(c[0, 0] - inv[i, i]) < 1e-7          # TestOptimizer.cpp:64-65
    (J,), _ = e.compute_covariances([[(VAR_CAM_INTR, 1), (VAR_CAM_INTR, 3), (VAR_CAM_INTR, 4)]], DAMPING)
    idx, rest = [1, 3, 4], [0, 2, 5]
    Hm = H[np.ix_(idx, idx)] - H[np.ix_(idx, rest)] @ np.linalg.solve(H[np.ix_(rest, rest)], H[np.ix_(rest, idx)])
    Jp = J[np.ix_([0, 4, 8], [0, 4, 8])]                 # parameter 0 of each variable
    assert np.linalg.norm(Hm @ Jp - np.eye(3)) < 1e-9   # TestOptimizer.cpp:81-82
    assert np.allclose(J, J.T, rtol=0, atol=1e-9 * np.abs(J).max())


def test_covariance_kat_oracle():
    from oracle.refcpu import RefEngine
    _kat(RefEngine)


def _blocks(p):
    """the SingleSessionProblem::computeCovariances request (SingleSessionProblem.cpp:66-118): per rig
    its pose, velocity and omega jointly (omega when it is estimated: with a second IMU); every calibration
    variable alone"""
    omega = len(p.fivals[4]) > 0
    blocks = [[(1, r), (2, r)] + ([(3, r)] if omega else []) for r in range(0, len(p.const[1]), 7)]
    for kind in (4, 5, 6, 7):
        blocks += [[(kind, h)] for h in range(len(p.const[kind])) if not p.const[kind][h]]
    return blocks


def test_covariances_oracle_symmetric_positive():
    from oracle.refcpu import RefEngine
    e, p = make(RefEngine, "A")
    covs, _ = e.compute_covariances(_blocks(p))
    for c in covs:
        assert np.allclose(c, c.T, atol=1e-12 * np.abs(c).max())
        assert np.linalg.eigvalsh(0.5 * (c + c.T)).min() > 0


@pytest.mark.gpu
def test_covariance_kat_gpu():
    from visual_inertial_bundle_adjustment_amd.engine import HipEngine
    _kat(HipEngine)


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["A", "miniB"])
def test_covariances_gpu_match_oracle(which):
    from oracle.refcpu import RefEngine
    from parity_util import rel
    from visual_inertial_bundle_adjustment_amd.engine import HipEngine, VbError
    g, p = make(HipEngine, which)
    r, _ = make(RefEngine, which)
    for e in (g, r):
        e.optimize(Settings.default(max_num_iterations=5))
    blocks = _blocks(p)
    cg, lg = g.compute_covariances(blocks)
    cr, lr = r.compute_covariances(blocks)
    assert lg == lr == DAMPING
    for a, b in zip(cg, cr):
        assert rel(a, b) < 1e-7
    # landmark points are eliminated by the engine; constant variables have no covariance
    with pytest.raises(VbError):
        g.compute_covariances([[(0, 0)]])
    with pytest.raises(VbError):
        g.compute_covariances([[(8, 0)]])
    # the LM state is rebuilt by the next iteration
    s = g.optimize(Settings.default(max_num_iterations=2))
    assert s.num_iterations == 2


def _all_blocks(p):
    """every rig block (pose, velocity, omega) and every calibration variable: the whole request of
    SingleSessionProblem::computeCovariances"""
    omega = len(p.fivals[4]) > 0
    blocks = [[(1, r), (2, r)] + ([(3, r)] if omega else []) for r in range(len(p.const[1]))]
    for kind in (4, 5, 6, 7):
        blocks += [[(kind, h)] for h in range(len(p.const[kind])) if not p.const[kind][h]]
    return blocks


def _solved(e, blocks, monkeypatch):
    """the same blocks by one reduced solve per column (VIBA_COV_SOLVES=1)"""
    monkeypatch.setenv("VIBA_COV_SOLVES", "1")
    try:
        return e.compute_covariances(blocks)
    finally:
        monkeypatch.delenv("VIBA_COV_SOLVES")


@pytest.mark.gpu
def test_selected_inversion_matches_column_solves_miniB(monkeypatch):
    """The selected inversion (csrc/selinv.hip) against one reduced solve per column on miniB, every
    rig and calibration block, plus joint blocks of far-apart rigs (off the factor's tile pattern: they
    take the per-column solves inside the same call)."""
    from parity_util import rel
    from visual_inertial_bundle_adjustment_amd.engine import HipEngine
    g, p = make(HipEngine, "miniB")
    g.optimize(Settings.default(max_num_iterations=3))
    n = len(p.const[1])
    blocks = _all_blocks(p) + [[(1, 0), (1, n - 1)], [(1, 3), (2, n // 2), (4, 0)]]
    ci, li = g.compute_covariances(blocks)
    cs, ls = _solved(g, blocks, monkeypatch)
    assert li == ls
    worst = max(rel(a, b) for a, b in zip(ci, cs))
    print(f"miniB: {len(blocks)} blocks, selected inversion vs column solves {worst:.2e}")
    assert worst < 1e-8
    for c in ci:
        assert np.allclose(c, c.T, rtol=0, atol=1e-10 * np.abs(c).max())


@pytest.mark.gpu
def test_selected_inversion_config_C_all_rigs(monkeypatch):
    """SingleSessionProblem::computeCovariances' whole request at config C (10k rig blocks of pose +
    velocity + omega, every calibration variable) in one call, in seconds; 40 sampled blocks against the
    per-column solves."""
    import time

    from parity_util import rel
    from visual_inertial_bundle_adjustment_amd import synth
    from visual_inertial_bundle_adjustment_amd.engine import HipEngine
    p = synth.generate(synth.config("C"))
    g = HipEngine(imu_calib_options=p.imu_calib_options)
    synth.load_into(g, p)
    blocks = _all_blocks(p)
    g.synchronize()
    t = time.perf_counter()
    ci, _ = g.compute_covariances(blocks)
    dt = time.perf_counter() - t
    print(f"config C: {len(blocks)} covariance blocks in {dt:.2f} s")
    assert dt < 20.0
    rng = np.random.default_rng(5)
    pick = sorted(rng.choice(len(blocks), size=40, replace=False))
    cs, _ = _solved(g, [blocks[i] for i in pick], monkeypatch)
    worst = max(rel(ci[i], c) for i, c in zip(pick, cs))
    print(f"config C: sampled blocks vs column solves {worst:.2e}")
    assert worst < 1e-8
    for c in ci[::97]:
        assert np.linalg.eigvalsh(0.5 * (c + c.T)).min() > 0
    g.close()
