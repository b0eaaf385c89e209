"""Matrix-free CPU oracle for grids too large for a host CSR -- TEST INFRASTRUCTURE ONLY.

Nothing in the product package (`helmholtz_preconditioner_amd`) imports this module; only
`tests/`, `__graft_entry__` and `bench.py`'s cpu_baseline leg may, as the checker.

It wraps oracle/stencil_oracle.c (built by oracle/Makefile, which __graft_entry__.build() runs):
the reference's operator row by row -- build_A_matrix's five entries per row (code.py:202-219),
coefficients by code.py:70-115 / 130-154, PML code.py:11-33, quirks Q3 / Q4 -- summed in scipy
csr_matvec's order, without storing the matrix (8192^2: 7 GB of CSR; 16384^2: 28 GB).  The solve
leg is still scipy's own gmres (code.py:516), given this operator as a LinearOperator; the
Jacobi M is 1 / diag(A) as oracle.jacobi_preconditioner forms it from A.diagonal().

Pinned in tests/test_oracle.py against oracle.helmholtz_oracle.build_A_matrix (itself pinned by
the reference's golden CSR / SpMV vectors) to rounding (<= 1e-15 relative), on every medium kind.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import scipy.sparse.linalg

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "build", "libhh_oracle.so")
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            raise ImportError(f"C oracle not built ({_LIB}): make -C oracle")
        _lib = ctypes.CDLL(_LIB)
        d = ctypes.c_double
        _lib.hho_apply.restype = ctypes.c_int
        _lib.hho_apply.argtypes = [ctypes.c_int, d, d, d, d, d, ctypes.c_void_p, d, d, d,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    return _lib


class MatrixFreeOperator(scipy.sparse.linalg.LinearOperator):
    """The operator of build_A_matrix(b, const, eta, omega, h, n, c_mat) (code.py:202) applied
    row by row in C.  c_mat: (n+2)^2 real array (read as c_mat[i-1, j-1], quirk Q3) or a
    positive scalar for a constant medium.  mass_scale multiplies omega^2 in the mass term
    (1 + i beta: the shifted operator build_A_matrix(c_mat / sqrt(1 + i beta)), to rounding)."""

    def __init__(self, b, const, eta, omega, h, n, c_mat, mass_scale=1.0):
        N = n * n
        super().__init__(dtype=np.complex128, shape=(N, N))
        self.n, self.const, self.eta, self.h = int(n), float(const), float(eta), float(h)
        self.omega, self.mass_scale = complex(omega), complex(mass_scale)
        if np.isscalar(c_mat):
            self.cc, self.c_const = None, float(c_mat)
        else:
            cm = np.asarray(c_mat, dtype=np.float64)
            # [j-1][i-1] = c_mat[i-1, j-1]: unit stride along the fast axis i (quirk Q3)
            self.cc, self.c_const = np.ascontiguousarray(cm[:n, :n].T), 0.0
        self._diag = None

    def _run(self, x, mode):
        y = np.empty(self.shape[0], dtype=np.complex128)
        xp = None
        if mode == 0:
            x = np.ascontiguousarray(np.ravel(x), dtype=np.complex128)
            xp = x.ctypes.data
        rc = _load().hho_apply(self.n, self.const, self.eta, self.omega.real, self.omega.imag,
                               self.h, None if self.cc is None else self.cc.ctypes.data,
                               self.c_const, self.mass_scale.real, self.mass_scale.imag, xp,
                               y.ctypes.data, mode)
        if rc != 0:
            raise RuntimeError(f"hho_apply failed ({rc})")
        return y

    def _matvec(self, x):
        y = self._run(x, 0)
        return y.reshape(-1, 1) if np.ndim(x) == 2 else y

    def diagonal(self):
        if self._diag is None:
            self._diag = self._run(None, 1)
        return self._diag


def jacobi_preconditioner(A):
    """M = diag(A)^-1 (oracle.helmholtz_oracle.jacobi_preconditioner's form)."""
    dinv = 1.0 / A.diagonal()
    N = A.shape[0]
    return scipy.sparse.linalg.LinearOperator((N, N), matvec=lambda x: dinv * np.ravel(x),
                                              dtype=np.complex128)
