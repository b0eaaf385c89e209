"""GPU tier, SURVEY row F4: the 9-point operator (``build_A_matrix(..., stencil=9)``) on the
HIP path against the oracle's restatement (``oracle.build_A9_matrix``).

The reference has no 9-point operator, so the oracle is pinned by properties
(tests/test_stencil9_oracle.py), not by reference outputs ("parity unpinned" by the
reference).  Tolerances as for the 5-point path: apply 1e-12 relative (norm-wise),
GMRES history and field 1e-6 (contract), CSR export bit-identical to the applied operator.
"""
import numpy as np
import pytest
import scipy.sparse
import scipy.sparse.linalg

import helmholtz_preconditioner_amd as H
from conftest import medium, rand_complex
from oracle import helmholtz_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-12
W9 = O.STENCIL9_WEIGHTS


@pytest.fixture(scope="module")
def ctx():
    c = H.Context(device=0)
    H.set_default_context(c)
    yield c
    H.set_default_context(None)


def relerr(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


def _op(n, kind, ctx, wn=5.0, weights=None, C=81.0):
    b = min(6, max(1, n // 3))
    om, h, eta = O.problem_params(n, b, wn, 2.0)
    cm = medium(kind, n) if isinstance(kind, str) else kind
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx, stencil=9, stencil_weights=weights)
    R = O.build_A9_matrix(b, C, eta, om, h, n, cm, weights=weights if weights else W9)
    return A, R


def test_default_weights_agree():
    assert tuple(H.STENCIL9_WEIGHTS) == tuple(W9)


@pytest.mark.parametrize("n,kind", [(1, "c1"), (2, "const"), (3, "c1"), (17, "c2"), (255, "c1"),
                                    (513, "const"), (700, "c2"), (1100, "c1"), (2100, "c1")])
def test_apply_vs_oracle(ctx, n, kind):
    """ragged sizes on every strip shape (256-wide below n = 2048, 512-wide above)"""
    A, R = _op(n, kind, ctx)
    assert A.stencil == 9
    for seed in range(2):
        x = rand_complex(n * n, seed)
        assert relerr(A @ x, R @ x) < TOL
    np.testing.assert_allclose(A.diagonal(), R.diagonal(), rtol=1e-13, atol=0)
    x = rand_complex(n * n, 5)
    yj = A._apply_host(x, H._ffi.HH_APPLY_JACOBI_A)
    assert relerr(yj, (R @ x) / R.diagonal()) < TOL


def test_unit_weights_equal_5pt_operator(ctx):
    n = 300
    A9, _ = _op(n, "c1", ctx, weights=(1.0, 1.0, 0.0))
    b = min(6, max(1, n // 3))
    om, h, eta = O.problem_params(n, b, 5.0, 2.0)
    A5 = H.build_A_matrix(b, 81.0, eta, om, h, n, medium("c1", n), context=ctx)
    x = rand_complex(n * n, 1)
    assert relerr(A9 @ x, A5 @ x) < 1e-14


def test_switching_stencil_on_one_operator(ctx):
    n = 129
    A, R9 = _op(n, "c1", ctx)
    b = min(6, max(1, n // 3))
    om, h, eta = O.problem_params(n, b, 5.0, 2.0)
    R5 = O.build_A_matrix(b, 81.0, eta, om, h, n, medium("c1", n))
    x = rand_complex(n * n, 2)
    assert relerr(A @ x, R9 @ x) < TOL
    A.set_stencil(5)
    assert relerr(A @ x, R5 @ x) < TOL
    A.set_stencil(9)
    assert relerr(A @ x, R9 @ x) < TOL


@pytest.mark.parametrize("slabs", [2, 3])
def test_virtual_slabs_bit_identical(slabs):
    n = 301
    outs = []
    for s in (1, slabs):
        c = H.Context(device=0, virtual_slabs=s)
        A, _ = _op(n, "c2", c)
        outs.append(A @ rand_complex(n * n, 4))
    np.testing.assert_array_equal(outs[0], outs[1])


def test_large_grid_properties(ctx):
    """4096^2, marmousi-like: linearity and A(x) vs the CSR the device exports (row sample)"""
    n = 4096
    om, h, eta = O.problem_params(n, 12, 100.0, 2.0)
    A = H.build_A_matrix(12, 81.0, eta, om, h, n, H.marmousi_like_c_mat(n), context=ctx, stencil=9)
    x, y = A.vector(), A.vector()
    x.fill_hash(11)
    A.apply_device(x, y)
    xa, ya = x.download(), y.download()
    z = A.vector(2.0 * xa)
    A.apply_device(z, y)
    np.testing.assert_array_equal(y.download(), 2.0 * ya)   # exact: scaling by 2
    rows = np.r_[0:3, n - 1:n + 2, 2048 * n + 5, n * n - n - 1:n * n]
    M = A.to_csr()
    assert M.nnz == (3 * n - 2) ** 2
    np.testing.assert_allclose((M[rows] @ xa), ya[rows], rtol=1e-13)


@pytest.mark.parametrize("n,kind", [(1, "const"), (2, "c1"), (5, "c1"), (64, "c2"), (300, "c1")])
def test_to_csr_vs_oracle(ctx, n, kind):
    A, R = _op(n, kind, ctx)
    M = A.to_csr()
    assert M.nnz == (3 * n - 2) ** 2 == R.nnz
    np.testing.assert_array_equal(M.indptr, R.indptr)
    np.testing.assert_array_equal(M.indices, R.indices)
    np.testing.assert_allclose(M.data, R.data, rtol=1e-13, atol=1e-13 * np.abs(R.data).max())
    x = rand_complex(n * n, 3)
    y = A @ x
    assert np.linalg.norm(M @ x - y) <= 1e-14 * np.linalg.norm(y)


def test_to_csr_slabs_bit_identical():
    n = 97
    outs = []
    for s in (1, 3):
        c = H.Context(device=0, virtual_slabs=s)
        A, _ = _op(n, "c1", c)
        outs.append(A.to_csr(index_dtype=np.int64))
    np.testing.assert_array_equal(outs[0].indptr, outs[1].indptr)
    np.testing.assert_array_equal(outs[0].indices, outs[1].indices)
    np.testing.assert_array_equal(outs[0].data, outs[1].data)


def _oracle_gmres(n, kind, M_kind, maxiter, rtol=1e-3, wn=4.0, beta=0.5, sweeps=2, damping=0.7):
    b = min(6, max(1, n // 3))
    om, h, eta = O.problem_params(n, b, wn, 2.0)
    cm = medium(kind, n)
    R = O.build_A9_matrix(b, 81.0, eta, om, h, n, cm)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    M = None
    if M_kind == "jacobi":
        M = O.jacobi_preconditioner(R)
    elif M_kind == "sl":
        Rb = O.build_A9_matrix(b, 81.0, eta, om, h, n, cm / np.sqrt(1 + 1j * beta))
        dinv = 1.0 / Rb.diagonal()

        def mv(r):
            r = np.ravel(r)
            z = damping * dinv * r
            for _ in range(sweeps - 1):
                z = z + damping * dinv * (r - Rb @ z)
            return z
        M = scipy.sparse.linalg.LinearOperator(R.shape, matvec=mv, dtype=np.complex128)
    return O.gmres_reference(R, f, M=M, rtol=rtol, restart=20, maxiter=maxiter), f


@pytest.mark.parametrize("M_kind,sweeps", [(None, 0), ("jacobi", 0), ("sl", 1), ("sl", 2), ("sl", 3)])
def test_gmres_vs_oracle(ctx, M_kind, sweeps):
    n = 64
    (xr, infor, histr, relr), f = _oracle_gmres(n, "c1", M_kind, 60, sweeps=max(sweeps, 1))
    A, _ = _op(n, "c1", ctx, wn=4.0)
    M = M_kind
    if M_kind == "sl":
        M = H.ShiftedLaplace(A, beta=0.5, sweeps=sweeps, damping=0.7)
    x, info, hist = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=60, M=M, callback=lambda r: None,
                            callback_type='legacy', return_history=True)
    assert info == infor and len(hist) == len(histr)
    assert np.max(np.abs(hist - histr) / histr) < 1e-6
    assert relerr(x, xr) < 1e-6


def test_gmres_converges_and_slabs_agree():
    """a converging 9-point solve (info 0) on 1 and 3 virtual slabs"""
    n = 40
    (xr, infor, histr, relr), f = _oracle_gmres(n, "c2", "jacobi", 400, rtol=1e-4, wn=1.0)
    assert infor == 0
    for s in (1, 3):
        c = H.Context(device=0, virtual_slabs=s)
        A, _ = _op(n, "c2", c, wn=1.0)
        x, info, hist = H.gmres(A, f, rtol=1e-4, restart=20, maxiter=400, M="jacobi",
                                callback=lambda r: None, callback_type='legacy',
                                return_history=True)
        assert info == 0 and len(hist) == len(histr)
        assert np.max(np.abs(hist - histr) / histr) < 1e-6
        assert relerr(x, xr) < 1e-6


def test_sweeping_refuses_9pt(ctx):
    A, _ = _op(48, "c1", ctx)
    with pytest.raises(H.HHError, match="5-point"):
        H.gmres(A, np.ones(48 * 48, complex), M=H.Sweeping(A), maxiter=2)
    A5, _ = _op(48, "c1", ctx)
    A5.set_stencil(5)
    A5.set_preconditioner(H._ffi.HH_PREC_SWEEP)
    with pytest.raises(H.HHError, match="5-point"):
        A5.set_stencil(9)


@pytest.mark.parametrize("n,kind", [(700, "c1"), (2100, "c2")])
def test_all_shapes_bit_identical(ctx, n, kind):
    """marching (256/512-wide, cached/NT) and tile (2 .. 8 rows) shapes of the 9-point apply and
    of its Jacobi-fused apply: identical numbers, and the oracle's"""
    A, R = _op(n, kind, ctx)
    x = rand_complex(n * n, 6)
    yref = R @ x
    first = firstj = None
    for v in (6, 18, 30, 42, 98, 99, 100, 101, 102, 104, 116, 132):
        A.tune(v, 0, 0)
        y = A @ x
        yj = A._apply_host(x, H._ffi.HH_APPLY_JACOBI_A)
        assert relerr(y, yref) < TOL, v
        first = y if first is None else first
        firstj = yj if firstj is None else firstj
        np.testing.assert_array_equal(y, first)
        np.testing.assert_array_equal(yj, firstj)
    A.tune(-1, 0, 0)
