"""Device Helmholtz operator: drop-in for the reference's ``build_A_matrix`` / ``A @ x``.

Reference (bocchs/helmholtz-preconditioner, code.py):
  build_A_matrix(b, const, eta, omega, h, n, c_mat) -> scipy sparse A   code.py:202-219
  A @ x   (scipy csr_matvec inside gmres, A passed at code.py:516)

Here ``build_A_matrix`` returns a :class:`DeviceOperator`, a
``scipy.sparse.linalg.LinearOperator`` whose matvec runs the hand-written gfx950
stencil kernel (helmholtz_preconditioner_amd/csrc/stencil.hip).  The CSR matrix is
never assembled: the operator holds 1-D PML tables and the pre-transposed 1/c^2
field of its row slab in HBM.  It therefore drops into
``scipy.sparse.linalg.gmres(A, f, ...)`` unchanged (each matvec is a host<->device
round trip), and into this package's device-resident :func:`gmres`.
"""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.sparse.linalg

from . import _ffi
from ._ffi import check, lib
from .context import Context, default_context

# Dispersion-optimal weights (alpha, c, d) of the 9-point operator (derived by
# tools/optimize_9pt.py: phase-velocity error <= 0.42 % at >= 4 points per wavelength).
STENCIL9_WEIGHTS = (0.7910350, 0.6276117, 0.0948567)


def _medium_arguments(c_mat, n):
    """Map the reference's c_mat to (host array | None, c_const, mass_scale).

    * real (n+2)^2 array -> streamed 1/c^2 field (or a constant medium when every
      entry is equal: then no 2-D field is stored or read);
    * complex c_mat = |c| * z with one phase z for every entry (the shifted-Laplace
      trick c_mat / sqrt(1 + i beta)) -> |c| field and mass scale 1/z^2, which gives the
      reference's omega^2 / (s1 s2 c_mat^2) exactly in exact arithmetic.
    """
    if int(n) < 1:
        raise ValueError(f"n must be >= 1 (got {n})")
    c = np.asarray(c_mat)
    if c.ndim != 2 or c.shape[0] < n + 2 or c.shape[1] < n + 2:
        raise ValueError(f"c_mat must be at least ({n + 2}, {n + 2}); got {c.shape}")
    # the reference reads c_mat[i-1, j-1] for i, j in 1..n only (code.py:108)
    used = c[:n, :n]
    mass = 1.0 + 0.0j
    if np.iscomplexobj(used):
        mag = np.abs(used)
        if np.any(mag == 0):
            raise ValueError("c_mat has zero entries")
        phase = used / mag
        z = phase.flat[0]
        if not np.allclose(phase, z, rtol=0, atol=1e-14):
            raise ValueError("complex c_mat must have a single common phase (c / sqrt(1 + i beta))")
        mass = 1.0 / (z * z)
        used = mag
        c = np.abs(c)
    used = np.asarray(used, dtype=np.float64)
    if np.all(used == used.flat[0]):
        return None, float(used.flat[0]), mass
    full = np.ascontiguousarray(np.asarray(c, dtype=np.float64)[: n + 2, : n + 2])
    return full, 0.0, mass


class DeviceVector:
    """A complex vector resident in HBM, laid out as this rank's slab of the operator."""

    def __init__(self, op: "DeviceOperator", data=None):
        self.op = op
        h = ctypes.c_void_p()
        check(lib.hh_vec_create(op.handle, ctypes.byref(h)))
        self._h = h
        _ffi.track(self, 0)
        if data is not None:
            self.upload(data)

    @property
    def handle(self):
        return self._h

    def upload(self, data):
        a = np.ascontiguousarray(np.ravel(data), dtype=np.complex128)
        if a.size != self.op.local_size:
            raise ValueError(f"expected {self.op.local_size} values, got {a.size}")
        check(lib.hh_vec_upload(self._h, _ffi.dptr(a)))

    def download(self):
        out = np.empty(self.op.local_size, dtype=np.complex128)
        check(lib.hh_vec_download(self._h, _ffi.dptr(out)))
        return out

    def fill_hash(self, seed: int = 0):
        check(lib.hh_vec_fill_hash(self._h, ctypes.c_uint64(seed)))

    def close(self):
        # the library keeps the operator (and its context) alive until its vectors are gone,
        # so a vector can always be released, whatever order a garbage collector picks
        if getattr(self, "_h", None) is not None:
            lib.hh_vec_destroy(self._h)
        self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class DeviceOperator(scipy.sparse.linalg.LinearOperator):
    """The PML Helmholtz operator A of code.py:202, applied matrix-free on the GPU.

    ``shape`` is (local, local): the whole N = n^2 system on a single rank, this
    rank's slab when the context spans several ranks.
    """

    def __init__(self, b, const, eta, omega, h, n, c_mat, context: Context | None = None,
                 stencil: int = 5, stencil_weights=None):
        self.ctx = context or default_context()
        self.b, self.const, self.eta, self.omega, self.h, self.n = b, const, eta, complex(omega), h, n
        host, c_const, mass = _medium_arguments(c_mat, n)
        self.constant_medium = host is None
        hnd = ctypes.c_void_p()
        check(lib.hh_op_create(self.ctx.handle, int(n), int(b), float(const), float(eta),
                               self.omega.real, self.omega.imag, float(h),
                               None if host is None else _ffi.dptr(host), float(c_const),
                               mass.real, mass.imag, ctypes.byref(hnd)))
        self._h = hnd
        _ffi.track(self, 1)
        jb, je = ctypes.c_int(), ctypes.c_int()
        check(lib.hh_op_local_rows(hnd, ctypes.byref(jb), ctypes.byref(je)))
        self.row_begin, self.row_end = jb.value, je.value
        self.local_size = (je.value - jb.value) * n
        self._precond = (_ffi.HH_PREC_NONE, 0.5, 1, 1.0)
        self.stencil, self.stencil_weights = 5, None
        if stencil != 5 or stencil_weights is not None:
            self.set_stencil(stencil, stencil_weights)
        super().__init__(dtype=np.complex128, shape=(self.local_size, self.local_size))

    def set_stencil(self, points: int = 9, weights=None):
        """Select the 5-point operator (the reference's, code.py:202-219) or the 9-point one
        (no reference counterpart): ``weights`` = (alpha, c, d), default
        :data:`STENCIL9_WEIGHTS`.  Applies, preconditioners, ``gmres`` and ``to_csr`` follow."""
        points = int(points)
        if points not in (5, 9):
            raise ValueError("stencil must be 5 or 9")
        w = tuple(float(v) for v in (weights if weights is not None else STENCIL9_WEIGHTS))
        if len(w) != 3:
            raise ValueError("stencil_weights must be (alpha, c, d)")
        check(lib.hh_op_set_stencil(self.handle, points, *w))
        self.stencil = points
        self.stencil_weights = w if points == 9 else None

    # ----------------------------------------------------------------- plumbing
    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("operator destroyed")
        return self._h

    @property
    def bytes_per_point(self) -> int:
        """Algorithmic HBM bytes of one apply per unknown."""
        return 32 if self.constant_medium else 40

    def set_preconditioner(self, kind: int, beta: float = 0.5, sweeps: int = 1, damping: float = 1.0):
        check(lib.hh_op_set_precond(self.handle, int(kind), float(beta), int(sweeps), float(damping)))
        self._precond = (kind, beta, sweeps, damping)

    def vector(self, data=None) -> DeviceVector:
        return DeviceVector(self, data)

    # ----------------------------------------------------------- LinearOperator
    def _apply_host(self, x, mode):
        x = np.asarray(x)
        shape = x.shape
        a = np.ascontiguousarray(np.ravel(x), dtype=np.complex128)
        if a.size != self.local_size:
            raise ValueError(f"dimension mismatch: {a.size} != {self.local_size}")
        y = np.empty_like(a)
        check(lib.hh_op_apply(self.handle, _ffi.dptr(a), _ffi.dptr(y), int(mode)))
        return y.reshape(shape)

    def _matvec(self, x):
        return self._apply_host(x, _ffi.HH_APPLY_A)

    def _rmatvec(self, x):
        # A is complex-symmetric (A^T == A), so A^H x = conj(A conj(x)).
        if self.stencil != 5:
            raise NotImplementedError("A^H of the 9-point operator (not symmetric): use to_csr()")
        return np.conj(self._apply_host(np.conj(x), _ffi.HH_APPLY_A))

    def _adjoint(self):
        return scipy.sparse.linalg.LinearOperator(self.shape, matvec=self._rmatvec,
                                                  rmatvec=self._matvec, dtype=self.dtype)

    def diagonal(self):
        """A.diagonal() of the local slab (c5 of code.py:107-109)."""
        d = np.empty(self.local_size, dtype=np.complex128)
        check(lib.hh_op_diagonal(self.handle, _ffi.dptr(d)))
        return d

    @property
    def csr_nnz(self) -> int:
        """Entries of this rank's rows in the assembled matrix (5 n^2 - 4 n on one rank;
        (3 n - 2)^2 for the 9-point operator)."""
        v = ctypes.c_int64()
        check(lib.hh_op_csr_nnz(self.handle, ctypes.byref(v)))
        return v.value

    def to_csr(self, index_dtype=None, return_kernel_ms: bool = False):
        """The scipy CSR matrix ``build_A_matrix`` returns (code.py:202-219), assembled on the
        device from the coefficients the stencil applies.

        One rank: the full N x N matrix, structurally identical to the reference's (canonical
        CSR, sorted columns S, W, D, E, N per row).  Several ranks: this rank's rows with
        global column indices, shape (local, N).  ``index_dtype`` defaults to int32 when
        N < 2^31 (scipy's choice), else int64.
        """
        import scipy.sparse
        N = self.n * self.n
        if index_dtype is None:
            index_dtype = np.int32 if N < 2 ** 31 else np.int64
        index_dtype = np.dtype(index_dtype)
        if index_dtype not in (np.dtype(np.int32), np.dtype(np.int64)):
            raise ValueError("index_dtype must be int32 or int64")
        nnz = self.csr_nnz
        indptr = np.empty(self.local_size + 1, dtype=np.int64)
        indices = np.empty(nnz, dtype=index_dtype)
        data = np.empty(nnz, dtype=np.complex128)
        ms = ctypes.c_double()
        check(lib.hh_op_export_csr(self.handle, indptr.ctypes.data_as(ctypes.c_void_p),
                                   indices.ctypes.data_as(ctypes.c_void_p), index_dtype.itemsize,
                                   _ffi.dptr(data), ctypes.byref(ms)))
        if index_dtype == np.dtype(np.int32):
            indptr = indptr.astype(np.int32)
        A = scipy.sparse.csr_matrix((data, indices, indptr), shape=(self.local_size, N),
                                    copy=False)
        if A.indices.dtype != index_dtype:  # scipy downcasts small matrices: keep the request
            A.indices, A.indptr = indices, indptr
        A.has_sorted_indices = True
        return (A, ms.value) if return_kernel_ms else A

    def apply_device(self, x: DeviceVector, y: DeviceVector, mode: int = _ffi.HH_APPLY_A):
        check(lib.hh_op_apply_dev(self.handle, x.handle, y.handle, int(mode)))

    def time_apply(self, x, y, iters: int, mode: int = _ffi.HH_APPLY_A):
        """(total_ms, avg stencil-kernel ms) over `iters` back-to-back device applies.
        ``x``/``y`` may be equal-length lists of DeviceVectors: apply i then maps
        x[i % len] -> y[i % len] (no apply re-reads what the previous one left in cache)."""
        xs = list(x) if isinstance(x, (list, tuple)) else [x]
        ys = list(y) if isinstance(y, (list, tuple)) else [y]
        if len(xs) != len(ys) or not xs:
            raise ValueError("x and y must be DeviceVectors or equal-length lists of them")
        raw = lambda v: v.handle.value if isinstance(v.handle, ctypes.c_void_p) else v.handle
        hx = (ctypes.c_void_p * len(xs))(*[raw(v) for v in xs])
        hy = (ctypes.c_void_p * len(ys))(*[raw(v) for v in ys])
        t, k = ctypes.c_double(), ctypes.c_double()
        check(lib.hh_op_time_apply_set(self.handle, hx, hy, len(xs), int(mode), int(iters),
                                       ctypes.byref(t), ctypes.byref(k)))
        return t.value, k.value

    def tune(self, variant: int = -1, rows_per_block: int = 0, grid_blocks: int = 0):
        """Select a stencil kernel variant / band height / persistent grid size (speed only;
        results are identical)."""
        check(lib.hh_op_tune(self.handle, int(variant), int(rows_per_block), int(grid_blocks)))

    def sl_fusion(self, enable: bool = True):
        """Two-sweep shifted-Laplace M: fused M A launch (default) or stencil + sweep pair
        (identical results; for A/B timing)."""
        check(lib.hh_op_sl_fusion(self.handle, int(bool(enable))))

    KRYLOV_MODES = {"auto": 0, "two": 1, "one": 2, "fused": 3}

    def krylov_mode(self, mode: str = "auto"):
        """GMRES inner-iteration form: "two" (projections, then the updated vector's norm --
        exact normalisation), "one" (lagged normalisation: one allreduce per iteration), "fused"
        ("one" with the update, the next M A and its projections in one pass over the basis,
        csrc/fused.hip: any slabs and ranks, 5-point operator, M none / Jacobi / the two-sweep
        shifted Laplace, restart <= 21), "auto" ("fused" where it applies and n >= 1024, else
        "one" across ranks and "two" on a single rank).  Results agree to rounding."""
        if mode not in self.KRYLOV_MODES:
            raise ValueError(f"mode must be one of {sorted(self.KRYLOV_MODES)}")
        check(lib.hh_op_set_krylov_mode(self.handle, self.KRYLOV_MODES[mode]))

    def small_cycle(self, mode: str = "auto"):
        """Whole-cycle GMRES kernel for small single-rank grids (csrc/gmres_small.hip): "auto"
        (where it applies and n^2 <= 2^18), "on" (wherever it applies), "off"."""
        modes = {"auto": -1, "off": 0, "on": 1}
        if mode not in modes:
            raise ValueError(f"mode must be one of {sorted(modes)}")
        check(lib.hh_op_set_small_cycle(self.handle, modes[mode]))

    def set_timing(self, enable: bool = True):
        """Diagnostic span timing (hh_op_set_timing): HIP events around the halo exchange,
        boundary / interior kernels, allreduces and Krylov kernels of the following applies
        and solves.  Adds queue work: for diagnostic runs only."""
        check(lib.hh_op_set_timing(self.handle, int(bool(enable))))

    def read_timing(self):
        """{span: (total ms, count)} since the last read (hh_op_read_timing)."""
        ms = np.zeros(len(_ffi.SPAN_NAMES))
        cnt = (ctypes.c_long * len(_ffi.SPAN_NAMES))()
        check(lib.hh_op_read_timing(self.handle, _ffi.dptr(ms), cnt))
        return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(_ffi.SPAN_NAMES)}

    SOLVE_PATHS = {0: "regular", 1: "small-cycle", 2: "small-cycle refused -> regular",
                   3: "one-pass"}

    def last_solve_path(self) -> str:
        """Cycle form the last ``gmres`` on this operator ran (hh_op_last_solve_path)."""
        p = ctypes.c_int(-1)
        check(lib.hh_op_last_solve_path(self.handle, ctypes.byref(p)))
        return self.SOLVE_PATHS[p.value]

    def stats(self):
        s = _ffi.HHStats()
        check(lib.hh_op_last_stats(self.handle, ctypes.byref(s)))
        return {f: getattr(s, f) for f, _ in _ffi.HHStats._fields_}

    def close(self):
        if getattr(self, "_h", None) is not None:
            lib.hh_op_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def build_A_matrix(b, const, eta, omega, h, n, c_mat, context: Context | None = None,
                   stencil: int = 5, stencil_weights=None):
    """Drop-in for ``build_A_matrix`` (code.py:202): same arguments, same operator.

    Returns a :class:`DeviceOperator` (a LinearOperator) instead of a scipy CSR
    matrix; ``A @ x`` / ``A.matvec(x)`` / ``A.diagonal()`` behave like the CSR's.
    ``stencil=9`` (keyword only, not in the reference) selects the 9-point operator
    (see :meth:`DeviceOperator.set_stencil`).
    """
    return DeviceOperator(b, const, eta, omega, h, n, c_mat, context=context, stencil=stencil,
                          stencil_weights=stencil_weights)


# ----------------------------------------------------------------- preconditioners
class DevicePreconditioner(scipy.sparse.linalg.LinearOperator):
    """An M for the reference's preconditioner slot (code.py:510-511) that runs on the
    device.  Pass it as ``M=`` to :func:`helmholtz_preconditioner_amd.gmres`; it is also
    a LinearOperator (host round trip) so ``scipy.sparse.linalg.gmres`` accepts it."""

    kind = _ffi.HH_PREC_NONE

    def __init__(self, A: DeviceOperator, beta=0.5, sweeps=1, damping=1.0):
        self.A, self.beta, self.sweeps, self.damping = A, beta, sweeps, damping
        super().__init__(dtype=np.complex128, shape=A.shape)

    def configure(self):
        self.A.set_preconditioner(self.kind, self.beta, self.sweeps, self.damping)

    def _matvec(self, x):
        self.configure()
        return self.A._apply_host(x, _ffi.HH_APPLY_PREC)


class Jacobi(DevicePreconditioner):
    """M = diag(A)^-1 (BASELINE config 2), fused into the stencil epilogue."""

    kind = _ffi.HH_PREC_JACOBI

    def __init__(self, A: DeviceOperator):
        super().__init__(A)


class ShiftedLaplace(DevicePreconditioner):
    """M ~= A_beta^-1, A_beta = build_A_matrix(..., c_mat / sqrt(1 + i beta)) (BASELINE
    config 3), approximated by `sweeps` damped-Jacobi sweeps from a zero guess."""

    kind = _ffi.HH_PREC_SHIFTED_LAPLACE

    def __init__(self, A: DeviceOperator, beta=0.5, sweeps=2, damping=0.7):
        super().__init__(A, beta, sweeps, damping)


class Sweeping(DevicePreconditioner):
    """The reference's own preconditioner: the sweeping moving-PML preconditioner
    (Engquist-Ying; algo2_3 / algo2_4, code.py:345-385), on the GPU.

    * ``reference=False`` (default): Algorithm 2.4 with the reference's bugs fixed --
      M x = sweep(x) (quirk Q1) and the middle sweep u_m = T_m u_m (quirk Q2).
    * ``reference=True``: exactly what run_solver runs (code.py:510-511): inside ``gmres``
      M x = algo2_4(b) for every x, middle sweep u_m -= T_m u_m.

    Setup factors H_F and all n - b moving-PML sub-problems H_m (b = the PML width passed
    to build_A_matrix) by block Thomas on the device.  Single rank, single slab only (the
    sweep is sequential in the layer index).
    """

    FORMS = {"auto": -1, "thomas": 0, "dense": 1, "dense-launches": 2, "thomas-sequential": 3}

    def __init__(self, A: DeviceOperator, reference: bool = False, form: str = "auto",
                 workgroups: int = 0):
        """``form``: ``"dense"`` forms the n matrices T_m (n^3 x 16 B of HBM) at setup and
        applies M as a chain of GEMVs; ``"thomas"`` keeps O(n^2 b^2) block-Thomas factors
        and solves, each forward / backward-sweep solve partitioned over 16 column chunks
        (3 x the factors' memory; sequential when that does not fit); ``"thomas-sequential"``
        the unpartitioned solves (2n dependent steps each, least memory); ``"auto"`` picks
        dense when n <= 2048 and it fits, else ``"thomas"``; ``"dense-launches"`` is the dense
        form with one launch per GEMV instead of the persistent chain (n <= 1024).  Same
        results to rounding (the two dense forms bit for bit).  ``workgroups``: how many
        workgroups share each partitioned solve (0: by n; ``hh_op_sweep_workgroups``)."""
        self.kind = _ffi.HH_PREC_SWEEP_REF if reference else _ffi.HH_PREC_SWEEP
        if form not in self.FORMS:
            raise ValueError(f"form must be one of {sorted(self.FORMS)}")
        self.form = form
        self.requested_workgroups = int(workgroups)
        super().__init__(A)

    def configure(self):
        A = self.A
        active, wgs = ctypes.c_int(), ctypes.c_int()
        check(lib.hh_op_sweep_workgroups(A.handle, self.requested_workgroups, ctypes.byref(wgs)))
        check(lib.hh_op_sweep_mode(A.handle, self.FORMS[self.form], ctypes.byref(active)))
        super().configure()
        check(lib.hh_op_sweep_mode(A.handle, self.FORMS[self.form], ctypes.byref(active)))
        check(lib.hh_op_sweep_workgroups(A.handle, self.requested_workgroups, ctypes.byref(wgs)))
        self.dense = active.value == 1
        self.partitioned = active.value == 2  # chunked block-Thomas solves
        self.workgroups = wgs.value  # workgroups per partitioned solve (0: not partitioned)
