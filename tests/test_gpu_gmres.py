"""GPU tier: the device-resident GMRES (csrc/krylov.hip + runtime.cpp) against the
reference solve (scipy gmres on the reference's CSR, golden vectors) and the oracle.

Tolerance (north star contract): residual history and field within 1e-6 relative.
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
    c = H.Context(device=0)
    H.set_default_context(c)
    yield c
    H.set_default_context(None)


def relerr(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


def _setup(z, ctx):
    n = int(z["n"])
    om = complex(z["omega"])
    A = H.build_A_matrix(int(z["b"]), float(z["C"]), float(z["eta"]), om, float(z["h"]), n,
                         medium(str(z["medium"]), n), context=ctx)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    return A, f


@pytest.mark.parametrize("name", ["gmres_n128_none.npz", "gmres_n128_jacobi.npz",
                                  "gmres_n64_c1_none.npz"])
@pytest.mark.parametrize("reorth", [False, True])
def test_gmres_matches_reference_golden(ctx, name, reorth):
    z = load_golden(name)
    A, f = _setup(z, ctx)
    M = "jacobi" if str(z["precond"]) == "jacobi" else None
    hist = []
    x, info = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=int(z["K"]), M=M,
                      callback=hist.append, callback_type='legacy', reorth=reorth)
    hist = np.array(hist)
    assert info == int(z["info"])
    assert len(hist) == int(z["niter"])
    assert np.max(np.abs(hist - z["history"]) / z["history"]) < TOL
    assert relerr(x, z["x"]) < TOL
    relres = np.linalg.norm(f - O.build_A_matrix(int(z["b"]), float(z["C"]), float(z["eta"]),
                                                 complex(z["omega"]), float(z["h"]), int(z["n"]),
                                                 medium(str(z["medium"]), int(z["n"]))) @ x) \
        / np.linalg.norm(f)
    assert abs(relres - float(z["relres"])) / float(z["relres"]) < TOL


def _oracle_solve(n, b, C, wn, al, cm, M_kind, rtol, restart, maxiter, x0=None, **kw):
    om, h, eta = O.problem_params(n, b, wn, al)
    Aref = O.build_A_matrix(b, C, eta, om, h, n, cm)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    M = None
    if M_kind == "jacobi":
        M = O.jacobi_preconditioner(Aref)
    elif M_kind == "sl":
        M, _ = O.shifted_laplace_jacobi(b, C, eta, om, h, n, cm, **kw)
    return O.gmres_reference(Aref, f, M=M, rtol=rtol, restart=restart, maxiter=maxiter, x0=x0), \
        (om, h, eta, f)


@pytest.mark.parametrize("sweeps", [1, 2, 4])
def test_gmres_shifted_laplace_vs_oracle(ctx, sweeps):
    n, b, C, wn, al = 64, 12, 81.0, 4.0, 2.0
    cm = medium("c1", n)
    (xr, infor, histr, relr), (om, h, eta, f) = _oracle_solve(
        n, b, C, wn, al, cm, "sl", 1e-3, 20, 80, beta=0.5, sweeps=sweeps, damping=0.7)
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    M = H.ShiftedLaplace(A, beta=0.5, sweeps=sweeps, damping=0.7)
    x, info, hist = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=80, M=M, callback=lambda r: None,
                            callback_type='legacy', return_history=True)
    assert info == infor and len(hist) == len(histr)
    assert np.max(np.abs(hist - histr) / histr) < TOL
    assert relerr(x, xr) < TOL


def test_gmres_converging_case_and_restart_cycles(ctx):
    """a small low-frequency problem that converges: info == 0, non-legacy maxiter
    (restart cycles), adaptive ptol path, x0 == 0"""
    n, b, C, wn, al = 40, 6, 61.0, 1.0, 2.0
    cm = medium("c2", n)
    (xr, infor, histr, relr), (om, h, eta, f) = _oracle_solve(n, b, C, wn, al, cm, "jacobi", 1e-4,
                                                                10, 400)
    assert infor == 0  # the oracle converges on this case
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    x, info, hist = H.gmres(A, f, rtol=1e-4, restart=10, maxiter=400, M="jacobi",
                            callback=lambda r: None, callback_type='legacy', return_history=True)
    assert info == 0
    assert len(hist) == len(histr)
    assert np.max(np.abs(hist - histr) / histr) < TOL
    assert relerr(x, xr) < TOL
    # callback None -> maxiter counts restart cycles (scipy semantics)
    x2, info2 = H.gmres(A, f, rtol=1e-4, restart=10, maxiter=400, M="jacobi")
    import scipy.sparse.linalg
    Aref = O.build_A_matrix(b, C, eta, om, h, n, cm)
    x3, info3 = scipy.sparse.linalg.gmres(Aref, f, rtol=1e-4, restart=10, maxiter=400,
                                          M=O.jacobi_preconditioner(Aref))
    assert info2 == info3 == 0
    assert relerr(x2, x3) < TOL


def test_gmres_nonzero_initial_guess(ctx):
    n, b, C, wn, al = 48, 6, 61.0, 2.0, 2.0
    cm = medium("c1", n)
    x0 = 1e-3 * rand_complex(n * n, 9)
    (xr, infor, histr, relr), (om, h, eta, f) = _oracle_solve(n, b, C, wn, al, cm, None, 1e-3, 20,
                                                                60, x0=x0.copy())
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    x, info, hist = H.gmres(A, f, x0=x0, rtol=1e-3, restart=20, maxiter=60,
                            callback=lambda r: None, callback_type='legacy', return_history=True)
    assert info == infor and len(hist) == len(histr)
    assert np.max(np.abs(hist - histr) / histr) < TOL
    assert relerr(x, xr) < TOL


def test_gmres_zero_rhs(ctx):
    n = 16
    om, h, eta = O.problem_params(n, 4, 2.0, 2.0)
    A = H.build_A_matrix(4, 61.0, eta, om, h, n, medium("const", n), context=ctx)
    x, info = H.gmres(A, np.zeros(n * n, complex), rtol=1e-3)
    assert info == 0 and not np.any(x)


@pytest.mark.parametrize("slabs", [2, 3])
def test_gmres_virtual_slabs_match_single_domain(slabs):
    """global inner products over slabs == single domain (fixed-order reductions)"""
    z = load_golden("gmres_n128_jacobi.npz")
    res = []
    for s in (1, slabs):
        c = H.Context(device=0, virtual_slabs=s)
        A, f = _setup(z, c)
        x, info, hist = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=60, M="jacobi",
                                callback=lambda r: None, callback_type='legacy',
                                return_history=True)
        res.append((x, hist))
    assert np.max(np.abs(res[1][1] - res[0][1]) / res[0][1]) < 1e-10
    assert relerr(res[1][0], res[0][0]) < 1e-10


def test_gmres_device_vectors_large(ctx):
    """config-3-shaped solve at n = 1024 through device vectors (no host round trip of
    N-vectors), one restart cycle, vs the oracle's scipy solve"""
    n, b, C, wn, al = 1024, 12, 81.0, 25.0, 2.0
    cm = H.marmousi_like_c_mat(n)
    (xr, infor, histr, relr), (om, h, eta, f) = _oracle_solve(
        n, b, C, wn, al, cm, "sl", 1e-12, 20, 20, beta=0.5, sweeps=2, damping=0.7)
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    bv = A.vector(f)
    xv, info, hist = H.gmres(A, bv, rtol=1e-12, restart=20, maxiter=20,
                             M=H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7),
                             callback=lambda r: None, callback_type='legacy', return_history=True)
    assert isinstance(xv, H.DeviceVector)
    assert np.max(np.abs(hist - histr) / histr) < TOL
    assert relerr(xv.download(), xr) < TOL


@pytest.mark.parametrize("ctype", ["x", "pr_norm"])
def test_gmres_callback_types_match_scipy(ctx, ctype):
    """callback_type='x' (the iterate after each restart cycle) and 'pr_norm' (per inner
    iteration; maxiter counts restart cycles) as scipy.sparse.linalg.gmres calls them."""
    import scipy.sparse.linalg
    n, b, C, wn, al = 40, 6, 61.0, 1.0, 2.0
    cm = medium("c2", n)
    om, h, eta = O.problem_params(n, b, wn, al)
    Aref = O.build_A_matrix(b, C, eta, om, h, n, cm)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    ref, got = [], []
    xr, infor = scipy.sparse.linalg.gmres(Aref, f, rtol=1e-5, restart=10, maxiter=8,
                                          M=O.jacobi_preconditioner(Aref),
                                          callback=lambda v: ref.append(np.copy(v)),
                                          callback_type=ctype)
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    x, info = H.gmres(A, f, rtol=1e-5, restart=10, maxiter=8, M="jacobi",
                      callback=lambda v: got.append(np.copy(v)), callback_type=ctype)
    assert info == infor and len(got) == len(ref) > 1
    if ctype == "x":
        for g, r in zip(got, ref):
            assert relerr(g, r) < 1e-6
    else:
        assert np.max(np.abs(np.array(got) - np.array(ref)) / np.array(ref)) < 1e-6
    assert relerr(x, xr) < 1e-6
