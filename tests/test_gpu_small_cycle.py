"""GPU tier: the whole-cycle GMRES kernel for small grids (csrc/gmres_small.hip; BASELINE
config 1 runs on it) against the reference's own histories (tests/golden: scipy gmres as
code.py:516 calls it) to the 1e-6 contract, and against the regular five-launch cycle.

Covered: config 1 itself (128^2, no preconditioner, K = 200 inner iterations: ten restart
cycles), Jacobi, a converging run (adaptive ptol, several cycles, info 0), nonzero x0, legacy
maxiter ending inside a cycle, restart 1 and 7, ragged n (block sizes not a multiple of the
wave, one-row grids), both media kinds.
"""
import numpy as np
import pytest

import helmholtz_preconditioner_amd as H
from conftest import load_golden, medium, rand_complex
from oracle import helmholtz_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope="module")
def ctx():
    return H.Context(device=0)


def relerr(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


@pytest.mark.parametrize("name", ["gmres_n128_none.npz", "gmres_n128_jacobi.npz",
                                  "gmres_n64_c1_none.npz"])
def test_small_cycle_matches_reference_golden(ctx, name):
    z = load_golden(name)
    n = int(z["n"])
    om = complex(z["omega"])
    A = H.build_A_matrix(int(z["b"]), float(z["C"]), float(z["eta"]), om, float(z["h"]), n,
                         medium(str(z["medium"]), n), context=ctx)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    M = "jacobi" if str(z["precond"]) == "jacobi" else None
    out = {}
    for mode in ("on", "off"):
        A.small_cycle(mode)
        hist = []
        x, info = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=int(z["K"]), M=M,
                          callback=hist.append, callback_type='legacy')
        out[mode] = (x, info, np.array(hist))
    A.small_cycle("auto")
    x, info, hist = out["on"]
    assert info == int(z["info"]) and len(hist) == int(z["niter"])
    assert np.max(np.abs(hist - z["history"]) / z["history"]) < TOL
    assert relerr(x, z["x"]) < TOL
    xo, _, ho = out["off"]  # (other summation order, lagged normalisation: rounding only)
    assert np.max(np.abs(hist - ho) / ho) < 1e-9
    assert relerr(x, xo) < 1e-9


@pytest.mark.parametrize("n,kind,precond,restart,K", [
    (37, "c1", None, 20, 45), (63, "c2", "jacobi", 7, 30), (65, "const", None, 1, 6),
    (1, "const", None, 20, 3), (2, "c1", "jacobi", 20, 3), (200, "c1", "jacobi", 20, 25),
    (128, "const", None, 23, 50)])
def test_small_cycle_matches_regular_cycle(ctx, n, kind, precond, restart, K):
    b, C, wn = min(6, max(1, n // 4)), 61.0, 3.0
    om, h, eta = O.problem_params(n, b, wn, 2.0)
    cm = medium(kind, n)
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    out = []
    for mode in ("on", "off"):
        A.small_cycle(mode)
        x, info, hist = H.gmres(A, f, rtol=1e-3, restart=restart, maxiter=K, M=precond,
                                callback=lambda r: None, callback_type="legacy",
                                return_history=True)
        out.append((x, info, hist))
    (x1, i1, h1), (x2, i2, h2) = out
    assert i1 == i2 and len(h1) == len(h2)
    assert np.all(np.abs(h1 - h2) <= 1e-9 * np.abs(h2) + 1e-15)  # (n = 1: presid 0)
    assert np.linalg.norm(x1 - x2) <= 1e-9 * np.linalg.norm(x2)


def test_small_cycle_converging_and_x0(ctx):
    n, b, C, wn, al = 40, 6, 61.0, 1.0, 2.0
    cm = medium("c2", n)
    om, h, eta = O.problem_params(n, b, wn, al)
    Aref = O.build_A_matrix(b, C, eta, om, h, n, cm)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    A.small_cycle("on")
    xr, infor, histr, _ = O.gmres_reference(Aref, f, M=O.jacobi_preconditioner(Aref), rtol=1e-4,
                                            restart=10, maxiter=400)
    x, info, hist = H.gmres(A, f, rtol=1e-4, restart=10, maxiter=400, M="jacobi",
                            callback=lambda r: None, callback_type='legacy', return_history=True)
    assert info == infor == 0 and len(hist) == len(histr)
    assert np.max(np.abs(hist - histr) / histr) < TOL
    assert relerr(x, xr) < TOL
    x0 = 1e-3 * rand_complex(n * n, 9)
    xr0, infor0, histr0, _ = O.gmres_reference(Aref, f, rtol=1e-3, restart=20, maxiter=60,
                                               x0=x0.copy())
    x5, info5, hist5 = H.gmres(A, f, x0=x0, rtol=1e-3, restart=20, maxiter=60,
                               callback=lambda r: None, callback_type='legacy',
                               return_history=True)
    assert info5 == infor0 and len(hist5) == len(histr0)
    assert np.max(np.abs(hist5 - histr0) / histr0) < TOL
    assert relerr(x5, xr0) < TOL
