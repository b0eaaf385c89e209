"""CPU oracle for the Helmholtz operator apply and GMRES solve.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package
(`helmholtz_preconditioner_amd`) imports this module.  Only `tests/`,
`__graft_entry__.smoke()` and the `cpu_baseline` leg of `bench.py` may use
it, and only as the checker / reported CPU baseline, never as the thing
measured or shipped.

What it is: a vectorised numpy/scipy restatement of the reference's hot path
(`/root/reference/code.py`, bocchs/helmholtz-preconditioner):

* PML profiles            sigma1/sigma2/s1/s2    code.py:11-33
* stencil coefficients    get_A_diag_block_coeffs code.py:70-115,
                          get_upper/lower_A_block code.py:130-154
* sparse assembly         get_A_block / build_A_matrix code.py:157-219
* apply                   ``A @ x`` (scipy csr_matvec; A passed at code.py:516)
* solve                   scipy.sparse.linalg.gmres(A, f, M=..., tol=...) code.py:516
  -- scipy is the reference's third-party dependency; the container pins
  scipy 1.15.3 (no requirements file in the reference).  The solve leg calls
  scipy's own gmres, with ``rtol=`` instead of the removed ``tol=``.
* inputs                  init_c1_mat/init_c2_mat/init_f1_mat/init_f2_mat code.py:39-66

Parity pinning: every function here is checked in ``tests/test_oracle.py``
against golden vectors in ``tests/golden/`` that were produced by importing
the reference ``code.py`` itself (script: ``tests/golden/make_golden.py``).

Quirks reproduced as-is:
  Q3  velocity read as c_mat[i-1, j-1] (transposed, shifted one cell),
  Q4  sigma2 is one-sided (PML only at x2 <= eta; Dirichlet top).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse
import scipy.sparse.linalg

__all__ = [
    "sigma1", "sigma2", "s1", "s2", "stencil_coefficients", "build_A_matrix",
    "init_c1_mat", "init_c2_mat", "init_f1_mat", "init_f2_mat",
    "jacobi_preconditioner", "shifted_laplace_jacobi", "gmres_reference",
    "problem_params", "slab_apply_emulated",
    "STENCIL9_WEIGHTS", "stencil9_coefficients", "build_A9_matrix", "phase_velocity_9pt",
    "coefficients_at", "apply_at_points",
]


# --------------------------------------------------------------------------
# PML profiles (code.py:11-33), vectorised.  Scalar branch logic kept exactly.
# --------------------------------------------------------------------------
def sigma1(x, const, eta):
    """Two-sided PML damping, code.py:11-18."""
    x = np.asarray(x, dtype=np.float64)
    lo = const / eta * ((x - eta) / eta) ** 2
    hi = const / eta * ((x - 1 + eta) / eta) ** 2
    return np.where(x <= eta, lo, np.where(x >= 1 - eta, hi, 0.0))


def sigma2(x, const, eta):
    """One-sided (bottom only) PML damping, code.py:20-25 (quirk Q4)."""
    x = np.asarray(x, dtype=np.float64)
    lo = const / eta * ((x - eta) / eta) ** 2
    return np.where(x <= eta, lo, 0.0)


def s1(x, const, eta, omega):
    """s1 = (1 + i*sigma1/omega)^-1, code.py:27-29."""
    return 1.0 / (1 + 1j * sigma1(x, const, eta) / omega)


def s2(x, const, eta, omega):
    """s2 = (1 + i*sigma2/omega)^-1, code.py:31-33."""
    return 1.0 / (1 + 1j * sigma2(x, const, eta) / omega)


# --------------------------------------------------------------------------
# Stencil coefficients.  Unknown p = (j-1)*n + (i-1); i is the fast axis
# (x1 = i*h), j the slow axis / layer (x2 = j*h)  -- code.py:81-113, 206-218.
# --------------------------------------------------------------------------
def coefficients_at(const, eta, omega, h, I, J, cc):
    """(W, E, S, N, D) at 1-based points (I, J) (arrays of one shape), with cc the velocity
    c_mat[i-1, j-1] there (quirk Q3 already applied by the caller); formulas of
    code.py:83-109.  The vectorised core of stencil_coefficients."""
    I = np.asarray(I, dtype=np.float64)
    J = np.asarray(J, dtype=np.float64)
    inv_h2 = 1 / h ** 2
    W = inv_h2 * (s1((I - .5) * h, const, eta, omega) / s2(J * h, const, eta, omega))
    E = inv_h2 * (s1((I + .5) * h, const, eta, omega) / s2(J * h, const, eta, omega))
    S = inv_h2 * (s2((J - .5) * h, const, eta, omega) / s1(I * h, const, eta, omega))
    N = inv_h2 * (s2((J + .5) * h, const, eta, omega) / s1(I * h, const, eta, omega))
    D = omega ** 2 / (s1(I * h, const, eta, omega) * s2(J * h, const, eta, omega) * cc ** 2) \
        - (W + E + S + N)
    return W, E, S, N, D


def stencil_coefficients(const, eta, omega, h, n, c_mat):
    """Return (W, E, S, N, D) as (n, n) complex arrays indexed [j-1, i-1].

    W = c1 (neighbour i-1), E = c2 (i+1), S = c3 (j-1), N = c4 (j+1),
    D = c5 (diagonal); formulas of code.py:83-109.  Coefficients of neighbours
    outside 1..n are returned too (they still enter D, code.py:107-109) but are
    dropped by the assembly.  ``c_mat`` is (n+2, n+2) real (or complex for the
    shifted-Laplace operator) and is read as c_mat[i-1, j-1] (quirk Q3).
    """
    idx = np.arange(1, n + 1, dtype=np.float64)
    I = idx[None, :]          # i along columns (fast axis)
    J = idx[:, None]          # j along rows   (slow axis)
    # c_mat[i-1, j-1] at (row j-1, col i-1) of our [j, i] layout -> transpose.
    cc = np.asarray(c_mat)[:n, :n].T
    return coefficients_at(const, eta, omega, h, I, J, cc)


def apply_at_points(const, eta, omega, h, n, c_of, x, P, stencil=5, weights=None):
    """(A x)[P] for flat 0-based indices P without assembling A (for grids too large to
    assemble on the host).  ``c_of(I, J)`` returns the velocity c_mat[i-1, j-1] at 1-based
    points; ``x`` is the full (n*n,) vector.  stencil=9 uses stencil9_coefficients' formulas
    (weights default STENCIL9_WEIGHTS)."""
    P = np.asarray(P, dtype=np.int64)
    J, I = P // n + 1, P % n + 1
    X = np.asarray(x)

    def u(di, dj):
        ii, jj = I + di, J + dj
        ok = (ii >= 1) & (ii <= n) & (jj >= 1) & (jj <= n)
        out = np.zeros(P.shape, dtype=np.complex128)
        out[ok] = X[(jj[ok] - 1) * n + (ii[ok] - 1)]
        return out

    if stencil == 5:
        W, E, S, N, D = coefficients_at(const, eta, omega, h, I, J, c_of(I, J))
        return S * u(0, -1) + W * u(-1, 0) + D * u(0, 0) + E * u(1, 0) + N * u(0, 1)
    co = _coef9(const, eta, omega, h, n, I, J, c_of(I, J), weights or STENCIL9_WEIGHTS)
    return sum(co[k] * u(di, dj) for k, di, dj in _OFF9)


def build_A_matrix(b, const, eta, omega, h, n, c_mat):
    """Global N x N CSR operator, same signature as code.py:202.

    Offsets {-n, -1, 0, +1, +n}; the +-1 entries are structurally absent at
    layer boundaries (block_diag of per-layer tridiagonals, code.py:213-218).
    ``b`` is unused by the assembly, exactly as in the reference.
    """
    W, E, S, N, D = stencil_coefficients(const, eta, omega, h, n, c_mat)
    NN = n * n
    lower1 = W[:, 1:]                     # entry (p, p-1) for i >= 2
    upper1 = E[:, :-1]                    # entry (p, p+1) for i <= n-1
    rows_l1 = (np.arange(n)[:, None] * n + np.arange(1, n)[None, :]).ravel()
    rows_u1 = (np.arange(n)[:, None] * n + np.arange(0, n - 1)[None, :]).ravel()
    rows_d = np.arange(NN)
    rows_ln = np.arange(n, NN)            # (p, p-n) for j >= 2 : coefficient S at row p
    rows_un = np.arange(0, NN - n)        # (p, p+n) for j <= n-1 : coefficient N at row p
    rows = np.concatenate([rows_ln, rows_l1, rows_d, rows_u1, rows_un])
    cols = np.concatenate([rows_ln - n, rows_l1 - 1, rows_d, rows_u1 + 1, rows_un + n])
    vals = np.concatenate([S[1:, :].ravel(), lower1.ravel(), D.ravel(), upper1.ravel(),
                           N[:-1, :].ravel()])
    A = scipy.sparse.csr_matrix((vals, (rows, cols)), shape=(NN, NN), dtype=np.complex128)
    A.sort_indices()
    return A


# --------------------------------------------------------------------------
# 9-point operator.  NO reference counterpart: the reference is 5-point
# only (code.py:216-218), so this restatement is pinned by properties, not by reference
# outputs ("parity unpinned" by the reference): it reduces to build_A_matrix exactly for
# weights (1, 1, 0), it is second-order consistent (the 3x3 weights of every symbol sum
# correctly), and its constant-medium dispersion matches phase_velocity_9pt.
#
#   A9 = alpha * A5_laplacian + (1 - alpha) * (line-averaged second differences)
#        + mass term M (c u_C + d sum(edges) + e sum(corners)),  e = (1 - c - 4d) / 4
# with the line-averaged part: the x second difference of code.py:83-106 averaged over
# rows j-1 and j+1 (with those rows' 1/s2 factor) and the y one over columns i-1, i+1.
# --------------------------------------------------------------------------
STENCIL9_WEIGHTS = (0.7910350, 0.6276117, 0.0948567)  # (alpha, c, d), tools/optimize_9pt.py


def _coef9(const, eta, omega, h, n, I, J, cc, weights):
    """the nine coefficients at 1-based points (I, J), cc = velocity there (see below)."""
    alpha, cw, dw = (float(v) for v in weights)
    g = (1.0 - alpha) / 2.0
    ew = (1.0 - cw - 4.0 * dw) / 4.0
    I = np.asarray(I, dtype=np.float64)
    J = np.asarray(J, dtype=np.float64)
    W, E, S, N, D = coefficients_at(const, eta, omega, h, I, J, cc)
    inv_h2 = 1 / h ** 2
    AW = inv_h2 * s1((I - .5) * h, const, eta, omega)
    AE = inv_h2 * s1((I + .5) * h, const, eta, omega)
    BS = inv_h2 * s2((J - .5) * h, const, eta, omega)
    BN = inv_h2 * s2((J + .5) * h, const, eta, omega)
    R2m = 1 / s2((J - 1) * h, const, eta, omega)
    R2p = 1 / s2((J + 1) * h, const, eta, omega)
    R1m = 1 / s1(np.maximum(I - 1, 1) * h, const, eta, omega)   # clamped like the kernel:
    R1p = 1 / s1(np.minimum(I + 1, n) * h, const, eta, omega)   # only multiplies ghosts
    M = omega ** 2 / (s1(I * h, const, eta, omega) * s2(J * h, const, eta, omega) * cc ** 2)
    Wm, Em, Wp, Ep = AW * R2m, AE * R2m, AW * R2p, AE * R2p
    Sm, Nm, Sp, Np = BS * R1m, BN * R1m, BS * R1p, BN * R1p
    return {
        "sw": g * (Wm + Sm) + ew * M, "s": alpha * S - g * (Wm + Em) + dw * M,
        "se": g * (Em + Sp) + ew * M, "w": alpha * W - g * (Sm + Nm) + dw * M,
        "c": cw * M - alpha * (W + E + S + N), "e": alpha * E - g * (Sp + Np) + dw * M,
        "nw": g * (Wp + Nm) + ew * M, "n": alpha * N - g * (Wp + Ep) + dw * M,
        "ne": g * (Ep + Np) + ew * M,
    }


def stencil9_coefficients(const, eta, omega, h, n, c_mat, weights=STENCIL9_WEIGHTS):
    """The nine coefficient arrays [j-1, i-1] of the 9-point operator, as a dict with keys
    sw, s, se, w, c, e, nw, n, ne (neighbour offsets (di, dj) = (-1,-1), (0,-1), ...).
    Entries for neighbours outside the grid are returned too; the assembly drops them."""
    idx = np.arange(1, n + 1, dtype=np.float64)
    cc = np.asarray(c_mat)[:n, :n].T
    return _coef9(const, eta, omega, h, n, idx[None, :], idx[:, None], cc, weights)


_OFF9 = (("sw", -1, -1), ("s", 0, -1), ("se", 1, -1), ("w", -1, 0), ("c", 0, 0),
         ("e", 1, 0), ("nw", -1, 1), ("n", 0, 1), ("ne", 1, 1))


def build_A9_matrix(b, const, eta, omega, h, n, c_mat, weights=STENCIL9_WEIGHTS):
    """Global CSR of the 9-point operator (same arguments as build_A_matrix, code.py:202):
    per row SW, S, SE, W, C, E, NW, N, NE where inside the grid; nnz = (3n-2)^2."""
    co = stencil9_coefficients(const, eta, omega, h, n, c_mat, weights)
    jj, ii = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    rows, cols, vals = [], [], []
    for key, di, dj in _OFF9:
        ok = (ii + di >= 0) & (ii + di < n) & (jj + dj >= 0) & (jj + dj < n)
        p = (jj * n + ii)[ok]
        rows.append(p)
        cols.append(p + dj * n + di)
        vals.append(co[key][ok])
    A = scipy.sparse.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                                shape=(n * n, n * n), dtype=np.complex128)
    A.sort_indices()
    return A


def phase_velocity_9pt(weights, G, phi):
    """Normalised numerical phase velocity of the constant-medium, PML-free 9-point scheme for
    a plane wave of G points per wavelength at angle phi (weights (1, 1, 0): the 5-point one).
    Symbol: alpha (2cos t + 2cos s - 4) + (1 - alpha)(4 cos t cos s - 2cos t - 2cos s)
            + (wh/c)^2 (c + 2d (cos t + cos s) + 4e cos t cos s) = 0."""
    alpha, cw, dw = weights
    ew = (1 - cw - 4 * dw) / 4
    kh = 2 * np.pi / np.asarray(G, dtype=np.float64)
    ct, cs = np.cos(kh * np.cos(phi)), np.cos(kh * np.sin(phi))
    L = alpha * (2 * ct + 2 * cs - 4) + (1 - alpha) * (4 * ct * cs - 2 * ct - 2 * cs)
    m = cw + 2 * dw * (ct + cs) + 4 * ew * ct * cs
    return np.sqrt(-L / m) / kh


# --------------------------------------------------------------------------
# Inputs (code.py:39-66)
# --------------------------------------------------------------------------
def init_c1_mat(r1, r2, n):
    x_i = np.linspace(0, 1, n + 2)
    xx, yy = np.meshgrid(x_i, x_i)
    return 4 / 3 * (1 - .5 * np.exp(-32 * ((xx - r1) ** 2 + (yy - r2) ** 2)))


def init_c2_mat(n):
    x_i = np.linspace(0, 1, n + 2)
    xx, yy = np.meshgrid(x_i, x_i)
    return 4 / 3 * (1 - .5 * np.exp(-32 * ((xx - .5) ** 2)))


def init_f1_mat(r1, r2, omega, n):
    x_i = np.linspace(0, 1, n + 2)
    xx, yy = np.meshgrid(x_i[1:-1], x_i[1:-1])
    return np.exp(-(4 * omega / np.pi) ** 2 * ((xx - r1) ** 2 + (yy - r2) ** 2))


def init_f2_mat(r1, r2, d1, d2, omega, n):
    x_i = np.linspace(0, 1, n + 2)
    xx, yy = np.meshgrid(x_i[1:-1], x_i[1:-1])
    return np.exp(-4 * omega * ((xx - r1) ** 2 + (yy - r2) ** 2)) \
        * np.exp(1j * omega * (xx * d1 + yy * d2))


def problem_params(n, b, wave_num, alpha):
    """omega, h, eta exactly as run_solver derives them (code.py:442-444)."""
    omega = 2 * np.pi * wave_num + 1j * alpha
    h = 1 / (n + 1)
    eta = b * h
    return omega, h, eta


# --------------------------------------------------------------------------
# Preconditioners filling the reference's M slot (code.py:510-511).
# --------------------------------------------------------------------------
def jacobi_preconditioner(A):
    """M = diag(A)^-1 as a LinearOperator (BASELINE config 2)."""
    dinv = 1.0 / A.diagonal()
    N = A.shape[0]
    return scipy.sparse.linalg.LinearOperator((N, N), matvec=lambda x: dinv * np.ravel(x),
                                              dtype=np.complex128)


def shifted_laplace_jacobi(b, const, eta, omega, h, n, c_mat, beta=0.5, sweeps=2,
                           damping=0.7):
    """Shifted-Laplace preconditioner M ~= A_beta^-1 (BASELINE config 3).

    A_beta = build_A_matrix(..., c_mat / sqrt(1 + i*beta)) -- the reference's own
    assembly with the complex-shifted mass term.  Its inverse
    is approximated by ``sweeps`` damped-Jacobi sweeps from a zero guess:
        z_0 = 0,  z_{k+1} = z_k + damping * D_beta^-1 (r - A_beta z_k).
    The first sweep is just damping*D^-1 r.  Must match the device kernel
    sequence (csrc/stencil.hip EPI_SL_FIRST / EPI_SL_SWEEP, and the fused two-sweep
    M A of csrc/sl_fused.hip): same recurrence, same order.  Default 2 sweeps, as in
    every graded path (BASELINE config 3, bench.py, driver.run_solver).
    """
    Ab = build_A_matrix(b, const, eta, omega, h, n, np.asarray(c_mat) / np.sqrt(1 + 1j * beta))
    dinv = 1.0 / Ab.diagonal()
    NN = n * n

    def mv(r):
        r = np.ravel(r)
        z = damping * dinv * r
        for _ in range(sweeps - 1):
            z = z + damping * dinv * (r - Ab @ z)
        return z

    return scipy.sparse.linalg.LinearOperator((NN, NN), matvec=mv, dtype=np.complex128), Ab


class _Counter:
    """gmres_counter of code.py:413-420 (counts legacy callbacks)."""

    def __init__(self):
        self.niter = 0
        self.history = []

    def __call__(self, rk=None):
        self.niter += 1
        self.history.append(float(rk))


def gmres_reference(A, b, M=None, rtol=1e-3, restart=20, maxiter=None, x0=None):
    """scipy.sparse.linalg.gmres exactly as code.py:516 calls it (legacy callback).

    Returns (x, info, presid_history, true_relres).  In legacy callback mode
    ``maxiter`` caps inner iterations (scipy iterative.py:792,820).
    """
    cnt = _Counter()
    x, info = scipy.sparse.linalg.gmres(A, b, x0=x0, rtol=rtol, restart=restart,
                                        maxiter=maxiter, M=M, callback=cnt,
                                        callback_type='legacy')
    relres = np.linalg.norm(b - A @ x) / np.linalg.norm(b)
    return x, info, np.array(cnt.history), relres


# --------------------------------------------------------------------------
# Row-slab decomposition emulator (test tier 4): P virtual slabs,
# each owning layers [j0, j1) with an explicit one-layer halo copy.
# --------------------------------------------------------------------------
def slab_apply_emulated(const, eta, omega, h, n, c_mat, x, bounds):
    """Apply A slab by slab with explicit halo copies; must equal A @ x."""
    W, E, S, N, D = stencil_coefficients(const, eta, omega, h, n, c_mat)
    X = np.asarray(x).reshape(n, n)
    out = []
    for (j0, j1) in bounds:                       # 0-based layer range
        loc = X[j0:j1]
        lo = X[j0 - 1] if j0 > 0 else np.zeros(n, X.dtype)      # halo from rank below
        hi = X[j1] if j1 < n else np.zeros(n, X.dtype)          # halo from rank above
        ext = np.vstack([lo[None], loc, hi[None]])
        y = D[j0:j1] * loc
        y[:, 1:] += W[j0:j1, 1:] * loc[:, :-1]
        y[:, :-1] += E[j0:j1, :-1] * loc[:, 1:]
        y += S[j0:j1] * ext[:-2] * (np.arange(j0, j1) > 0)[:, None]
        y += N[j0:j1] * ext[2:] * (np.arange(j0, j1) < n - 1)[:, None]
        out.append(y)
    return np.vstack(out).ravel()


# --------------------------------------------------------------------------
# Sweeping moving-PML preconditioner: get_Hm_coeffs code.py:222-279,
# get_Hm code.py:283-290, get_A_FF/Fb1/b1F code.py:177-199, algo2_3 code.py:345-353,
# algo2_4 code.py:356-385.  SuperLU via scipy.sparse.linalg.splu as the reference.
# --------------------------------------------------------------------------
def s2m(x, m, b, const, eta, omega, h):
    """Moving-PML stretch s2 shifted to the bottom of sub-domain m, code.py:35-37."""
    return 1.0 / (1 + 1j * sigma2(np.asarray(x) - (m - b) * h, const, eta) / omega)


def hm_matrix(m, b, const, eta, omega, h, n, c_mat):
    """H_m (b n x b n) for 1-based m: layers j = m-b+1..m with the moving PML, code.py:222-290."""
    I = np.arange(1, n + 1, dtype=np.float64)[None, :]
    J = np.arange(m - b + 1, m + 1, dtype=np.float64)[:, None]
    inv_h2 = 1 / h ** 2
    sm = lambda x: s2m(x, m, b, const, eta, omega, h)  # noqa: E731
    W = inv_h2 * (s1((I - .5) * h, const, eta, omega) / sm(J * h))
    E = inv_h2 * (s1((I + .5) * h, const, eta, omega) / sm(J * h))
    S = inv_h2 * (sm((J - .5) * h) / s1(I * h, const, eta, omega))
    N = inv_h2 * (sm((J + .5) * h) / s1(I * h, const, eta, omega))
    cc = np.asarray(c_mat)[:n, m - b:m].T           # c_mat[i-1, j-1], rows j
    D = omega ** 2 / (s1(I * h, const, eta, omega) * sm(J * h) * cc ** 2) - (W + E + S + N)
    bn = b * n
    c1 = W.ravel()[1:].copy()
    c2 = E.ravel()[:-1].copy()
    c1[n - 1::n] = 0
    c2[n - 1::n] = 0
    A = scipy.sparse.diags([D.ravel(), c1, c2, S.ravel()[n:], N.ravel()[:-n]],
                           [0, -1, 1, -n, n], shape=(bn, bn), format='csc')
    return A


class SweepState:
    """algo2_3 setup + the coupling blocks run_solver prepares (code.py:496-507)."""

    def __init__(self, b, const, eta, omega, h, n, c_mat):
        self.b, self.n = b, n
        W, E, S, N, D = stencil_coefficients(const, eta, omega, h, n, c_mat)
        # A_FF = block_diag(A_11 .. A_bb): per-layer tridiagonals, no inter-layer blocks
        blocks = []
        for k in range(b):
            blocks.append(scipy.sparse.diags([D[k], W[k, 1:], E[k, :-1]], [0, -1, 1]))
        self.lu_HF = scipy.sparse.linalg.splu(scipy.sparse.block_diag(blocks, format='csc'))
        self.lu_Hm = [scipy.sparse.linalg.splu(hm_matrix(m, b, const, eta, omega, h, n, c_mat))
                      for m in range(b + 1, n + 1)]
        self.S, self.N = S, N          # S[k]: A_{k+1,k} (0-based layers), N[k]: A_{k,k+1}

    def T(self, m, v):
        """lu_Hm.solve([0 .. 0, v])[-n:] for 1-based m."""
        tmp = np.zeros(self.b * self.n, complex)
        tmp[-self.n:] = v
        return self.lu_Hm[m - self.b - 1].solve(tmp)[-self.n:]

    def apply(self, f, corrected=False):
        """algo2_4 applied to f (as-is: quirk Q2 in the middle sweep; corrected: u_m = T_m u_m)."""
        b, n = self.b, self.n
        u = np.array(np.asarray(f).reshape(n, n), dtype=complex)
        TFuF = self.lu_HF.solve(u[:b].ravel())
        u[b] = u[b] - self.S[b] * TFuF[-n:]
        for m in range(b + 1, n):
            u[m] = u[m] - self.S[m] * self.T(m, u[m - 1])
        uF = TFuF
        for m in range(b + 1, n + 1):
            t = self.T(m, u[m - 1])
            u[m - 1] = t if corrected else u[m - 1] - t
        for m in range(n - 1, b, -1):
            u[m - 1] = u[m - 1] - self.T(m, self.N[m - 1] * u[m])
        Au = np.zeros(b * n, complex)
        Au[-n:] = self.N[b - 1] * u[b]
        uF = uF - self.lu_HF.solve(Au)
        u[:b] = uF.reshape(b, n)
        return u.ravel()


def sweeping_preconditioner(b, const, eta, omega, h, n, c_mat, f=None, corrected=False):
    """M for the gmres slot: as-is (code.py:510-511, quirk Q1) M x = algo2_4(f) for every x;
    corrected: M x = algo2_4(x) with the Alg. 2.4 middle sweep."""
    st = SweepState(b, const, eta, omega, h, n, c_mat)
    NN = n * n
    if corrected:
        mv = lambda x: st.apply(np.ravel(x), corrected=True)  # noqa: E731
    else:
        fixed = st.apply(np.ravel(f))
        mv = lambda x: fixed.copy()  # noqa: E731
    return scipy.sparse.linalg.LinearOperator((NN, NN), matvec=mv, dtype=np.complex128), st
