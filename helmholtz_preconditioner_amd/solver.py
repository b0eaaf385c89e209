"""Device-resident restarted GMRES: drop-in for the reference's solve call.

Reference: ``u, exit_code = scipy.sparse.linalg.gmres(A, f_vec, M=M, tol=1e-3,
callback=counter)`` at code.py:516 (scipy 1.15.3 ``_isolve/iterative.py:582-840``;
``tol=`` is spelled ``rtol=`` since scipy 1.14).  Same signature, same return
``(x, info)``, same control flow (left preconditioning, restart cycles, the
gh-8400 inner tolerance, legacy callback counting, true-residual outer test) --
but every N-vector operation runs in HBM on the GPU (csrc/krylov.hip) and the
host only sees per-iteration scalars.
"""
from __future__ import annotations

import ctypes
import warnings

import numpy as np

from . import _ffi
from ._ffi import check, lib
from .operator import DeviceOperator, DevicePreconditioner, DeviceVector, Jacobi


def _resolve_precond(A: DeviceOperator, M):
    if M is None:
        A.set_preconditioner(_ffi.HH_PREC_NONE)
        return
    if isinstance(M, str):
        if M.lower() == "jacobi":
            M = Jacobi(A)
        else:
            raise ValueError(f"unknown preconditioner {M!r}")
    if isinstance(M, DevicePreconditioner):
        if M.A is not A:
            raise ValueError("preconditioner was built for a different operator")
        M.configure()
        return
    raise TypeError(
        "device gmres accepts M=None, 'jacobi', Jacobi(A), ShiftedLaplace(A) or Sweeping(A); an "
        "arbitrary host LinearOperator M cannot run on the device -- use "
        "scipy.sparse.linalg.gmres(A, b, M=M) with this DeviceOperator instead")


def gmres(A, b, x0=None, *, rtol=1e-5, atol=0., restart=None, maxiter=None, M=None,
          callback=None, callback_type=None, reorth=False, return_history=False):
    """scipy.sparse.linalg.gmres semantics on a :class:`DeviceOperator`.

    ``b``/``x0`` may be numpy arrays (this rank's slab) or :class:`DeviceVector`s.
    Returns ``(x, info)`` (numpy x for numpy b, DeviceVector otherwise); with
    ``return_history=True`` also the per-iteration relative preconditioned
    residuals (what a legacy callback receives).
    """
    if not isinstance(A, DeviceOperator):
        raise TypeError("A must be a DeviceOperator from build_A_matrix")
    if callback is not None and callback_type is None:
        warnings.warn("scipy.sparse.linalg.gmres called without specifying `callback_type`. "
                      "The default value will be changed in a future release.",
                      category=DeprecationWarning, stacklevel=2)
    if callback_type is None:
        callback_type = 'legacy'
    if callback_type not in ('x', 'pr_norm', 'legacy'):
        raise ValueError(f"Unknown callback_type: {callback_type!r}")
    if callback is None:
        callback_type = None
    # scipy's defaults are taken on the GLOBAL system size N = n^2 (iterative.py: n =
    # len(b)), not on this rank's slab: every rank then runs the same number of cycles and
    # collectives, whatever the slab sizes.
    N = int(A.n) * int(A.n)
    if restart is None:
        restart = 20
    restart = min(restart, N)
    if maxiter is None:
        maxiter = N * 10
    legacy = callback_type == 'legacy'

    _resolve_precond(A, M)
    host_in = not isinstance(b, DeviceVector)
    bv = A.vector(np.asarray(b).ravel()) if host_in else b
    if x0 is None:
        xv = A.vector()
    elif isinstance(x0, DeviceVector):
        xv = x0
    else:
        xv = A.vector(np.asarray(x0).ravel())

    cap = maxiter if legacy else maxiter * restart
    cap = int(min(cap, 1 << 22))
    hist = np.zeros(max(cap, 1), dtype=np.float64)
    cb = _ffi.GMRES_CALLBACK(0)
    hcb = _ffi.GMRES_HISTORY_CALLBACK(0)
    ccb = _ffi.GMRES_CYCLE_CALLBACK(0)
    # An exception raised by the user's callback propagates out of gmres, as in scipy: the
    # trampoline stores it and returns non-zero, hh_gmres stops at once (HH_ERR_ABORTED), and
    # the stored exception is re-raised here (ctypes would otherwise print and drop it).
    raised = []
    if callback is not None and callback_type in ('legacy', 'pr_norm'):
        # one foreign call per restart cycle (hh_op_set_history_callback), the user's callback
        # still once per inner iteration, in order, where scipy calls it
        def _hcb(_user, _first, count, rel):
            for i, r in enumerate(rel[:count]):  # (one conversion of the cycle's values)
                try:
                    callback(r)
                except BaseException as e:  # noqa: BLE001 -- re-raised after hh_gmres returns
                    raised.append(e)
                    return i + 1
            return 0
        hcb = _ffi.GMRES_HISTORY_CALLBACK(_hcb)
    elif callback is not None:  # 'x': the iterate after every restart cycle (downloaded for
        def _ccb(_user, _cycle):  # numpy b, the DeviceVector itself otherwise)
            try:
                callback(xv.download() if host_in else xv)
            except BaseException as e:  # noqa: BLE001
                raised.append(e)
                return 1
            return 0
        ccb = _ffi.GMRES_CYCLE_CALLBACK(_ccb)
    iters, info, rnorm, bnorm = ctypes.c_long(), ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
    check(lib.hh_op_set_cycle_callback(A.handle, ccb, None))
    check(lib.hh_op_set_history_callback(A.handle, hcb, None))
    try:
        rc = lib.hh_gmres(A.handle, bv.handle, xv.handle, float(rtol), float(atol),
                          int(restart), int(maxiter), int(legacy), int(bool(reorth)),
                          _ffi.dptr(hist), cap, cb, None, ctypes.byref(iters),
                          ctypes.byref(info), ctypes.byref(rnorm), ctypes.byref(bnorm))
        if rc == _ffi.HH_ERR_ABORTED and raised:
            raise raised[0]
        check(rc)
    finally:
        check(lib.hh_op_set_cycle_callback(A.handle, _ffi.GMRES_CYCLE_CALLBACK(0), None))
        check(lib.hh_op_set_history_callback(A.handle, _ffi.GMRES_HISTORY_CALLBACK(0), None))
    A.last_solve = dict(iterations=iters.value, info=info.value, rnorm=rnorm.value,
                        bnorm=bnorm.value, stats=A.stats())
    x = xv.download() if host_in else xv
    out = (x, info.value)
    if return_history:
        out = out + (hist[: min(iters.value, cap)].copy(),)
    return out
