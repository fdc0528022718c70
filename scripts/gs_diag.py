"""Gauss-Seidel pseudo-factor breakdown probe: assemble the damped reduced system of miniB on the GPU,
copy the tile store to the host and check every diagonal tile's Cholesky with numpy; then the GPU's own
pseudo-factor (damp_factor_solve with the Gauss-Seidel solver) at the same lambdas."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from parity_util import make  # noqa: E402
from visual_inertial_bundle_adjustment_amd.engine import HipEngine, VbError  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "miniB"
hip = C.CDLL("libamdhip64.so")
TS = 64


def tiles_host(e):
    m, ml, r, rl = C.c_void_p(), C.c_int64(), C.c_void_p(), C.c_int64()
    e._check(e._fn("reduced_buffers", [C.POINTER(C.c_void_p), C.POINTER(C.c_int64), C.POINTER(C.c_void_p),
                                       C.POINTER(C.c_int64)])(e.h, C.byref(m), C.byref(ml), C.byref(r), C.byref(rl)))
    out = np.zeros(ml.value)
    assert hip.hipDeviceSynchronize() == 0
    assert hip.hipMemcpy(out.ctypes.data_as(C.c_void_p), m, C.c_size_t(ml.value * 8), 2) == 0
    return out.reshape(-1, TS, TS), rl.value // TS


def slot(e, i, j):
    s = C.c_int64()
    e._check(e._fn("debug_tile_slot", [C.c_int32, C.c_int32, C.POINTER(C.c_int64)])(e.h, i, j, C.byref(s)))
    return s.value


for lam in (1e-5, 1e-2, 1.0):
    e, _ = make(HipEngine, which)
    e.linearize(True, False)
    e._check(e._fn("assemble_reduced", [C.c_double])(e.h, lam))
    T, nT = tiles_host(e)
    bad = []
    for J in range(nT):
        A = T[slot(e, J, J)].T  # column-major tile -> row index first
        L = np.tril(A)
        S = L + np.tril(A, -1).T
        ev = np.linalg.eigvalsh(S)
        try:
            np.linalg.cholesky(S)
        except np.linalg.LinAlgError:
            bad.append((J, ev[0], ev[-1], float(np.abs(A - A.T).max())))
        if J < 3 or ev[0] <= 0:
            print(f"lam {lam:g} tile {J}: eig [{ev[0]:.3e}, {ev[-1]:.3e}] diag min {np.diag(S).min():.3e} "
                  f"upper-vs-lower asym {np.abs(np.triu(A, 1) - np.tril(A, -1).T).max():.3e}", flush=True)
    print(f"lam {lam:g}: {nT} diagonal tiles, numpy Cholesky fails on {len(bad)}: {bad[:5]}", flush=True)
    for solver in (0, 3):
        g, _ = make(HipEngine, which)
        if solver:
            g.set_solver(solver, 40, 1e-10)
        g.linearize(True, False)
        try:
            m = g.damp_factor_solve(lam)
            print(f"lam {lam:g} solver {solver}: ok, model reduction {m:.6e}", flush=True)
        except VbError as ex:
            print(f"lam {lam:g} solver {solver}: {ex}", flush=True)
