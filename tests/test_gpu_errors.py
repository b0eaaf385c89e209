"""GPU tier: error behaviour of the boundary (include/helmholtz_amd.h through the ctypes shim).

The reference raises Python exceptions (scipy's ValueError on shape mismatches, numpy errors);
the build raises ValueError / TypeError in the shim for what it can check on the host, and
HHError (a negative hh_err with hh_last_error()'s message) for what the C library rejects.
After any rejected call the objects stay usable.
"""
import numpy as np
import pytest
import scipy.sparse.linalg

import helmholtz_preconditioner_amd as H
from conftest import medium, rand_complex
from oracle import helmholtz_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = H.Context(device=0)
    H.set_default_context(c)
    yield c
    H.set_default_context(None)


@pytest.fixture(scope="module")
def op(ctx):
    n = 40
    om, h, eta = O.problem_params(n, 6, 3.0, 2.0)
    A = H.build_A_matrix(6, 81.0, eta, om, h, n, medium("c1", n), context=ctx)
    R = O.build_A_matrix(6, 81.0, eta, om, h, n, medium("c1", n))
    return A, R, (om, h, eta)


def _still_works(A, R):
    x = rand_complex(A.shape[0], 1)
    assert np.linalg.norm(A @ x - R @ x) <= 1e-12 * np.linalg.norm(R @ x)


def test_bad_operator_arguments(ctx):
    om, h, eta = O.problem_params(8, 2, 3.0, 2.0)
    with pytest.raises(ValueError, match="n must be"):
        H.build_A_matrix(2, 81.0, eta, om, h, 0, np.ones((2, 2)), context=ctx)
    with pytest.raises(ValueError, match="c_mat must be"):
        H.build_A_matrix(2, 81.0, eta, om, h, 8, np.ones((5, 5)), context=ctx)
    cm = np.ones((10, 10), complex)
    cm[0, 0] = 1j
    with pytest.raises(ValueError, match="single common phase"):
        H.build_A_matrix(2, 81.0, eta, om, h, 8, cm, context=ctx)
    with pytest.raises(H.HHError, match="positive"):
        H.build_A_matrix(2, 81.0, 0.0, om, h, 8, np.ones((10, 10)), context=ctx)
    with pytest.raises(ValueError, match="stencil must be 5 or 9"):
        H.build_A_matrix(2, 81.0, eta, om, h, 8, np.ones((10, 10)), context=ctx, stencil=7)


def test_bad_apply_and_vector_shapes(op):
    A, R, _ = op
    with pytest.raises(ValueError, match="dimension mismatch"):
        A @ np.ones(A.shape[0] + 1, complex)
    with pytest.raises(ValueError, match="expected"):
        A.vector(np.ones(3, complex))
    x, y = A.vector(), A.vector()
    with pytest.raises(ValueError):
        A.time_apply([x, y], [y], 2)
    with pytest.raises(H.HHError, match="distinct"):
        A.time_apply(x, x, 2)
    _still_works(A, R)


def test_bad_solver_arguments(op):
    A, R, (om, h, eta) = op
    f = np.ones(A.shape[0], complex)
    with pytest.raises(H.HHError, match="restart must be"):
        H.gmres(A, f, restart=40, maxiter=2)
    with pytest.raises(ValueError, match="unknown preconditioner"):
        H.gmres(A, f, M="ilu", maxiter=2)
    with pytest.raises(TypeError, match="host LinearOperator"):
        H.gmres(A, f, M=scipy.sparse.linalg.aslinearoperator(R), maxiter=2)
    B = H.build_A_matrix(6, 81.0, eta, om, h, A.n, medium("c1", A.n))
    with pytest.raises(ValueError, match="different operator"):
        H.gmres(A, f, M=H.Jacobi(B), maxiter=2)
    with pytest.raises(ValueError, match="Unknown callback_type"):
        H.gmres(A, f, callback=lambda r: None, callback_type="nope", maxiter=2)
    with pytest.raises(ValueError, match="expected"):
        H.gmres(A, f[:-1], maxiter=2)
    with pytest.raises(TypeError):
        H.gmres(R, f, maxiter=2)
    # the operator and the solver still work after every rejection
    x, info, hist = H.gmres(A, f, rtol=1e-3, maxiter=5, callback=lambda r: None,
                            callback_type="legacy", return_history=True)
    xr, infor, histr, _ = O.gmres_reference(R, f, rtol=1e-3, maxiter=5)
    assert info == infor and np.max(np.abs(hist - histr) / histr) < 1e-6
    _still_works(A, R)


def test_bad_tuning_and_preconditioner_settings(op):
    A, R, _ = op
    with pytest.raises(H.HHError, match="not instantiated"):
        A.tune(999)
    with pytest.raises(H.HHError, match="sweeps must be"):
        A.set_preconditioner(H._ffi.HH_PREC_SHIFTED_LAPLACE, 0.5, 0, 0.7)
    with pytest.raises(H.HHError, match="unknown preconditioner kind"):
        A.set_preconditioner(17)
    A.tune(-1)
    A.set_preconditioner(H._ffi.HH_PREC_NONE)
    _still_works(A, R)


def test_sweeping_needs_one_slab():
    c = H.Context(device=0, virtual_slabs=2)
    n = 32
    om, h, eta = O.problem_params(n, 6, 3.0, 2.0)
    A = H.build_A_matrix(6, 81.0, eta, om, h, n, medium("c1", n), context=c)
    with pytest.raises(H.HHError, match="one rank and one slab"):
        H.gmres(A, np.ones(n * n, complex), M=H.Sweeping(A), maxiter=2)
    R = O.build_A_matrix(6, 81.0, eta, om, h, n, medium("c1", n))
    _still_works(A, R)


class _Stop(Exception):
    pass


def _raise_at(k):
    calls = []

    def cb(r):
        calls.append(r)
        if len(calls) == k:
            raise _Stop(f"stop at {k}")
    return cb, calls


@pytest.mark.parametrize("callback_type", ["legacy", "pr_norm", "x"])
def test_callback_exception_propagates(op, callback_type):
    """scipy propagates an exception raised by the callback out of gmres (users rely on it
    to stop a solve early); the device solve stops at once and re-raises it."""
    A, R, _ = op
    f = np.ones(A.shape[0], complex)
    cb, calls = _raise_at(3 if callback_type != "x" else 1)
    with pytest.raises(_Stop):
        H.gmres(A, f, rtol=1e-12, restart=5, maxiter=50, callback=cb, callback_type=callback_type)
    assert len(calls) == (3 if callback_type != "x" else 1)
    # nothing of the aborted solve is left behind: plain applies and a new solve are exact
    _still_works(A, R)
    x, info, hist = H.gmres(A, f, rtol=1e-3, maxiter=5, callback=lambda r: None,
                            callback_type="legacy", return_history=True)
    xr, infor, histr, _ = O.gmres_reference(R, f, rtol=1e-3, maxiter=5)
    assert info == infor and np.max(np.abs(hist - histr) / histr) < 1e-6


@pytest.mark.parametrize("small", ["on", "off"])
def test_per_iteration_and_history_callbacks_agree(op, small):
    """hh_gmres's per-iteration callback (raw ABI) and the batched history callback the shim
    uses receive the same values in the same order; a stop request from either ends the solve
    with HH_ERR_ABORTED at the iteration it names"""
    import ctypes
    F = H._ffi
    A, R, _ = op
    A.small_cycle(small)
    f = np.ones(A.shape[0], complex)
    bv, maxiter = A.vector(f), 23

    def run(per_it_stop=0, hist_stop=0):
        xv = A.vector()
        per, batch = [], []

        def _cb(_u, it, rel):
            per.append((it, rel))
            return 1 if it == per_it_stop else 0

        def _hcb(_u, first, count, rel):
            for i in range(count):
                batch.append((first + i, rel[i]))
                if first + i == hist_stop:
                    return i + 1
            return 0
        cb, hcb = F.GMRES_CALLBACK(_cb), F.GMRES_HISTORY_CALLBACK(_hcb)
        F.check(F.lib.hh_op_set_history_callback(A.handle, hcb, None))
        hist = np.zeros(maxiter)
        it, info = ctypes.c_long(), ctypes.c_int()
        rn, bn = ctypes.c_double(), ctypes.c_double()
        try:
            rc = F.lib.hh_gmres(A.handle, bv.handle, xv.handle, 1e-12, 0.0, 5, maxiter, 1, 0,
                                F.dptr(hist), maxiter, cb, None, ctypes.byref(it),
                                ctypes.byref(info), ctypes.byref(rn), ctypes.byref(bn))
        finally:
            F.check(F.lib.hh_op_set_history_callback(A.handle, F.GMRES_HISTORY_CALLBACK(0),
                                                     None))
        return rc, it.value, per, batch, hist

    rc, it, per, batch, hist = run()
    assert rc == 0 and it == maxiter
    assert per == batch and [p[0] for p in per] == list(range(1, maxiter + 1))
    assert np.array_equal(np.array([p[1] for p in per]), hist)
    rc, it, per, batch, _ = run(per_it_stop=7)
    assert rc == F.HH_ERR_ABORTED and it == 7 and len(per) == 7
    rc, it, per, batch, _ = run(hist_stop=8)
    assert rc == F.HH_ERR_ABORTED and it == 8 and batch[-1][0] == 8
    A.small_cycle("auto")
    _still_works(A, R)


def test_aborted_asis_sweep_leaves_no_constant_map(ctx):
    """Sweeping(reference=True) makes M a constant map (algo2_4(b), quirk Q1) for the
    duration of a solve only: after a solve aborted by its callback, a plain M x is
    algo2_4(x) again (the in-solve state is released on every exit path)."""
    n, b, C = 37, 6, 61.0
    om, h, eta = O.problem_params(n, b, 3.0, 2.0)
    cm = medium("c2", n)
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    M = H.Sweeping(A, reference=True)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    cb, _ = _raise_at(1)
    with pytest.raises(_Stop):
        H.gmres(A, f, rtol=1e-12, maxiter=50, M=M, callback=cb, callback_type="legacy")
    st = O.SweepState(b, C, eta, om, h, n, cm)
    x = rand_complex(n * n, 5)
    want = st.apply(x)
    got = M @ x
    assert np.linalg.norm(got - want) <= 1e-10 * np.linalg.norm(want)
    R = O.build_A_matrix(b, C, eta, om, h, n, cm)
    _still_works(A, R)


def test_default_maxiter_and_restart_follow_the_global_size(op):
    """scipy's defaults restart = min(20, N) and maxiter = 10 N use the global N = n^2."""
    A, R, _ = op
    f = np.ones(A.shape[0], complex)
    c, cr = [], []
    x, info = H.gmres(A, f, rtol=1e-3, callback=c.append, callback_type="legacy")
    xr, infor = scipy.sparse.linalg.gmres(R, f, rtol=1e-3, callback=cr.append,
                                          callback_type="legacy")
    # this solve runs for hundreds of iterations, far past the horizon where scipy's own run is
    # reproducible to 1e-6: both must converge the same way, not bit for bit
    assert info == infor == 0 and abs(len(c) - len(cr)) <= 0.05 * len(cr), (len(c), len(cr))
    for u in (x, xr):
        assert np.linalg.norm(f - R @ u) <= 1e-3 * np.linalg.norm(f)
    assert np.linalg.norm(x - xr) <= 1e-3 * np.linalg.norm(xr)
    np.testing.assert_allclose(c[:10], cr[:10], rtol=1e-6)
