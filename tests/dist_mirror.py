"""Distributed GMRES mirror over torch.distributed (gloo, CPU) -- test helper.

Restates, in numpy, what the C runtime does at world > 1 (runtime.cpp run_stencil /
hh_gmres with the RCCL transport): each rank owns the layer slab
[floor(r n / P), floor((r+1) n / P)) (dist.slab_bounds), applies the stencil after a
one-row halo exchange with its neighbours, and forms every inner product as local partial
sums + an allreduce; the Hessenberg / Givens scalars are then identical on every rank and
drive scipy's control flow (restart cycles, legacy counting, ptol, true-residual test).
Classical Gram-Schmidt with lazily applied basis scales, like csrc/krylov.hip.
"""
import numpy as np
import torch
import torch.distributed as dist
from scipy.linalg import get_lapack_funcs

from oracle import helmholtz_oracle as O


class SlabOperator:
    def __init__(self, const, eta, omega, h, n, c_mat, j0, j1, jacobi=False, stencil=5):
        W, E, S, N, D = O.stencil_coefficients(const, eta, omega, h, n, c_mat)
        self.W, self.E, self.S, self.N, self.D = (a[j0:j1] for a in (W, E, S, N, D))
        self.co9 = None
        if stencil == 9:  # the same one-row halo carries the corner neighbours
            co = O.stencil9_coefficients(const, eta, omega, h, n, c_mat)
            self.co9 = {k: v[j0:j1] for k, v in co.items()}
            self.D = self.co9["c"]
        self.n, self.j0, self.j1 = n, j0, j1
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.jacobi = jacobi
        self.halo_calls = 0  # halo exchanges so far (gmres_dist_onepass counts them per pass)

    def _halo(self, X):
        self.halo_calls += 1
        n = self.n
        lo, hi = np.zeros(n, complex), np.zeros(n, complex)
        reqs = []
        buf_lo = torch.zeros(2 * n, dtype=torch.float64)
        buf_hi = torch.zeros(2 * n, dtype=torch.float64)
        if self.rank > 0:
            reqs.append(dist.isend(torch.from_numpy(X[0].view(np.float64).copy()), self.rank - 1))
            reqs.append(dist.irecv(buf_lo, self.rank - 1))
        if self.rank < self.world - 1:
            reqs.append(dist.isend(torch.from_numpy(X[-1].view(np.float64).copy()), self.rank + 1))
            reqs.append(dist.irecv(buf_hi, self.rank + 1))
        for r in reqs:
            r.wait()
        if self.rank > 0:
            lo = buf_lo.numpy().view(np.complex128).copy()
        if self.rank < self.world - 1:
            hi = buf_hi.numpy().view(np.complex128).copy()
        return lo, hi

    def apply(self, x):
        X = x.reshape(-1, self.n)
        lo, hi = self._halo(X)
        ext = np.vstack([lo[None], X, hi[None]])
        if self.co9 is not None:
            m, c = X.shape[0], self.co9
            y = np.zeros_like(X)
            for dj, (kw, kc, ke) in ((-1, ("sw", "s", "se")), (0, ("w", "c", "e")),
                                     (1, ("nw", "n", "ne"))):
                R = ext[1 + dj:1 + dj + m]
                y[:, 1:] += c[kw][:, 1:] * R[:, :-1]
                y += c[kc] * R
                y[:, :-1] += c[ke][:, :-1] * R[:, 1:]
            return y.ravel()
        y = self.S * ext[:-2]
        y[:, 1:] += self.W[:, 1:] * X[:, :-1]
        y += self.D * X
        y[:, :-1] += self.E[:, :-1] * X[:, 1:]
        y += self.N * ext[2:]
        return y.ravel()

    def psolve(self, r):
        return r / self.D.ravel() if self.jacobi else r.copy()


def allreduce(vals):
    t = torch.from_numpy(np.ascontiguousarray(vals, dtype=np.float64).copy())
    dist.all_reduce(t)
    return t.numpy()


def gdot(a, b):  # global vdot(a, b)
    v = np.vdot(a, b)
    s = allreduce([v.real, v.imag])
    return s[0] + 1j * s[1]


def gnorm(a):
    return float(np.sqrt(allreduce([np.vdot(a, a).real])[0]))


def gmres_dist(op, b, rtol, restart, maxiter):
    """legacy-callback GMRES (maxiter = inner iterations); returns (x, info, history)."""
    lartg = get_lapack_funcs('lartg', dtype=np.complex128)
    eps = np.finfo(float).eps
    x = np.zeros_like(b)
    bn = gnorm(b)
    atol = rtol * bn
    Mb = gnorm(op.psolve(b))
    ptol_f = 1.0
    ptol = Mb * min(ptol_f, atol / bn)
    V = np.empty((restart + 1, b.size), complex)
    scale = np.zeros(restart + 1)
    H = np.zeros((restart, restart + 1), complex)
    G = np.zeros((restart, 2), complex)
    hist, inner = [], 0
    r = b.copy()
    presid = 0.0
    for _ in range(maxiter):
        V[0] = op.psolve(r)
        t = gnorm(V[0])
        scale[0] = 1 / t
        S = np.zeros(restart + 1, complex)
        S[0] = t
        brk = False
        for col in range(restart):
            w = scale[col] * op.psolve(op.apply(V[col]))
            raw = allreduce(np.concatenate([[c.real, c.imag] for c in (V[:col + 1].conj() @ w)]
                                           + [[np.vdot(w, w).real]]))
            dots = raw[0:2 * (col + 1):2] + 1j * raw[1:2 * (col + 1):2]
            h0 = np.sqrt(raw[-1])
            hk = scale[:col + 1] * dots
            w = w - (hk * scale[:col + 1]) @ V[:col + 1]
            h1 = gnorm(w)
            H[col, :col + 1] = hk
            H[col, col + 1] = h1
            V[col + 1] = w
            if h1 <= eps * h0:
                H[col, col + 1] = 0
                brk = True
            else:
                scale[col + 1] = 1 / h1
            for k in range(col):
                c, s = G[k]
                n0, n1 = H[col, [k, k + 1]]
                H[col, [k, k + 1]] = [c * n0 + s * n1, -s.conj() * n0 + c * n1]
            c, s, mag = lartg(H[col, col], H[col, col + 1])
            G[col] = [c, s]
            H[col, [col, col + 1]] = mag, 0
            tmp = -np.conj(s) * S[col]
            S[[col, col + 1]] = [c * S[col], tmp]
            presid = abs(tmp)
            inner += 1
            hist.append(presid / bn)
            if inner == maxiter or presid <= ptol or brk:
                break
        if H[col, col] == 0:
            S[col] = 0
        y = S[:col + 1].copy()
        for k in range(col, 0, -1):
            if y[k] != 0:
                y[k] /= H[k, k]
                y[:k] -= y[k] * H[k, :k]
        if y[0] != 0:
            y[0] /= H[0, 0]
        x += (y * scale[:col + 1]) @ V[:col + 1]
        r = b - op.apply(x)
        rn = gnorm(r)
        if inner == maxiter:
            return x, (0 if rn <= atol else maxiter), np.array(hist)
        if rn <= atol or brk:
            break
        ptol_f = max(eps, 0.25 * ptol_f) if presid <= ptol else min(1.0, 1.5 * ptol_f)
        ptol = presid * min(ptol_f, atol / rn)
    return x, (0 if rn <= atol else maxiter), np.array(hist)


_COUNT = {"allreduce": 0}


def counted_allreduce(vals):
    _COUNT["allreduce"] += 1
    return allreduce(vals)


def gmres_dist_lagged(op, b, rtol, restart, maxiter):
    """The one-allreduce inner iteration of csrc/krylov.hip gmres_lag_kernel (the runtime's
    default across ranks), restated: raw basis u_k with exact norms sigma_k learned one
    iteration late (the norm of the vector an update wrote travels with the next iteration's
    projections), SpMV inputs scaled by the Pythagorean estimate meanwhile.  Returns
    (x, info, history, allreduces per inner iteration inside the cycles' loops -- the last
    column's norm adds one per cycle)."""
    lartg = get_lapack_funcs('lartg', dtype=np.complex128)
    eps = np.finfo(float).eps
    x = np.zeros_like(b)
    bn = gnorm(b)
    atol = rtol * bn
    Mb = gnorm(op.psolve(b))
    ptol_f = 1.0
    ptol = Mb * min(ptol_f, atol / bn)
    U = np.empty((restart + 1, b.size), complex)
    vs = np.zeros(restart + 1)   # exact 1 / sigma_k
    ss = np.zeros(restart + 1)   # SpMV input scales
    H = np.zeros((restart, restart + 1), complex)
    G = np.zeros((restart, 2), complex)
    hist, inner, cycle_reduces = [], 0, 0
    r = b.copy()
    presid = 0.0
    for _ in range(maxiter):
        U[0] = op.psolve(r)
        t = gnorm(U[0])
        vs[0] = ss[0] = 1 / t
        S = np.zeros(restart + 1, complex)
        S[0] = t
        brk = False
        h0 = {}
        stop_col = min(restart - 1, maxiter - inner - 1)

        def finish(col, h1):
            nonlocal brk, presid
            H[col, col + 1] = h1
            if h1 <= eps * h0[col]:
                H[col, col + 1] = 0
                brk = True
            for k in range(col):
                c, s = G[k]
                n0, n1 = H[col, [k, k + 1]]
                H[col, [k, k + 1]] = [c * n0 + s * n1, -s.conj() * n0 + c * n1]
            c, s, mag = lartg(H[col, col], H[col, col + 1])
            G[col] = [c, s]
            H[col, [col, col + 1]] = mag, 0
            tmp = -np.conj(s) * S[col]
            S[[col, col + 1]] = [c * S[col], tmp]
            presid = abs(tmp)
            hist.append(presid / bn)
            return presid <= ptol or brk or col >= stop_col

        col, done = -1, False
        for j in range(stop_col + 1):
            w = ss[j] * op.psolve(op.apply(U[j]))
            loc = [np.vdot(U[k], w) for k in range(j + 1)]
            vals = sum(([c.real, c.imag] for c in loc), []) + [np.vdot(w, w).real]
            if j > 0:
                vals.append(np.vdot(U[j], U[j]).real)   # the previous update's vector
            raw = counted_allreduce(vals)
            cycle_reduces += 1
            d = raw[0:2 * (j + 1):2] + 1j * raw[1:2 * (j + 1):2]
            w2 = raw[2 * (j + 1)]
            if j > 0:
                sj = np.sqrt(raw[2 * (j + 1) + 1])
                f = vs[j - 1] / ss[j - 1]
                vs[j] = 1 / sj
                col = j - 1
                if finish(col, sj * f):
                    done = True
                    break
            f = vs[j] / ss[j]
            H[j, :j + 1] = d * vs[:j + 1] * f
            h0[j] = np.sqrt(w2) * f
            ss[j + 1] = 1 / np.sqrt(max(w2 - np.sum(np.abs(d) ** 2 * vs[:j + 1] ** 2),
                                        max(w2 * 1e-28, 1e-300)))
            U[j + 1] = w - (d * vs[:j + 1] ** 2) @ U[:j + 1]
        if not done:  # the cycle's last column: one more (per-cycle) reduction
            sl = np.sqrt(counted_allreduce([np.vdot(U[stop_col + 1], U[stop_col + 1]).real])[0])
            col = stop_col
            vs[stop_col + 1] = 1 / sl
            finish(col, sl * vs[col] / ss[col])
        inner += col + 1
        if H[col, col] == 0:
            S[col] = 0
        y = S[:col + 1].copy()
        for k in range(col, 0, -1):
            if y[k] != 0:
                y[k] /= H[k, k]
                y[:k] -= y[k] * H[k, :k]
        if y[0] != 0:
            y[0] /= H[0, 0]
        x += (y * vs[:col + 1]) @ U[:col + 1]
        r = b - op.apply(x)
        rn = gnorm(r)
        if inner == maxiter:
            return x, (0 if rn <= atol else maxiter), np.array(hist), cycle_reduces / inner
        if rn <= atol or brk:
            break
        ptol_f = max(eps, 0.25 * ptol_f) if presid <= ptol else min(1.0, 1.5 * ptol_f)
        ptol = presid * min(ptol_f, atol / rn)
    return x, (0 if rn <= atol else maxiter), np.array(hist), cycle_reduces / inner


def gmres_dist_onepass(op, b, rtol, restart, maxiter):
    """The one-pass inner iteration across ranks (csrc/runtime.cpp run_fused + hh_gmres, DESIGN
    3g), restated in the runtime's order: a cycle starts with w_0 = M A (s_0 u_0) and its
    projection (one allreduce); then every pass K forms u_K = w_{K-1} - sum_k c_k u_k on the
    rank's own rows, exchanges ONLY u_K's edge rows (fused_edge_kernel + the halo exchange: the
    neighbours' passes read them as their halo rows), forms w_K = M A (s_K u_K) from the own rows
    and the received ones, and reduces <u_k, w_K> (k <= K), |w_K|^2 and |u_K|^2 in ONE allreduce;
    the cycle's last update adds one allreduce (its norm).  Same Hessenberg arithmetic as
    gmres_dist_lagged.  Returns (x, info, history, allreduces per pass, halo exchanges per pass):
    each pass is one inner iteration's update + M A + projection."""
    lartg = get_lapack_funcs('lartg', dtype=np.complex128)
    eps = np.finfo(float).eps
    x = np.zeros_like(b)
    bn = gnorm(b)
    atol = rtol * bn
    Mb = gnorm(op.psolve(b))
    ptol_f = 1.0
    ptol = Mb * min(ptol_f, atol / bn)
    U = np.empty((restart + 1, b.size), complex)
    vs = np.zeros(restart + 1)
    ss = np.zeros(restart + 1)
    H = np.zeros((restart, restart + 1), complex)
    G = np.zeros((restart, 2), complex)
    hist, inner, reduces, halos, passes = [], 0, 0, 0, 0
    r = b.copy()
    presid = 0.0
    for _ in range(maxiter):
        U[0] = op.psolve(r)
        t = gnorm(U[0])
        vs[0] = ss[0] = 1 / t
        S = np.zeros(restart + 1, complex)
        S[0] = t
        brk = False
        h0 = {}
        stop_col = min(restart - 1, maxiter - inner - 1)

        def finish(col, h1):
            nonlocal brk, presid
            H[col, col + 1] = h1
            if h1 <= eps * h0[col]:
                H[col, col + 1] = 0
                brk = True
            for k in range(col):
                c, s = G[k]
                n0, n1 = H[col, [k, k + 1]]
                H[col, [k, k + 1]] = [c * n0 + s * n1, -s.conj() * n0 + c * n1]
            c, s, mag = lartg(H[col, col], H[col, col + 1])
            G[col] = [c, s]
            H[col, [col, col + 1]] = mag, 0
            tmp = -np.conj(s) * S[col]
            S[[col, col + 1]] = [c * S[col], tmp]
            presid = abs(tmp)
            hist.append(presid / bn)
            return presid <= ptol or brk or col >= stop_col

        def start(j, d, w2):  # column j from the raw dots; the next SpMV input's scale
            f = vs[j] / ss[j]
            H[j, :j + 1] = d * vs[:j + 1] * f
            h0[j] = np.sqrt(w2) * f
            ss[j + 1] = 1 / np.sqrt(max(w2 - np.sum(np.abs(d) ** 2 * vs[:j + 1] ** 2),
                                        max(w2 * 1e-28, 1e-300)))

        # the cycle's head: w_0 and its projection
        w = ss[0] * op.psolve(op.apply(U[0]))
        raw = counted_allreduce([np.vdot(U[0], w).real, np.vdot(U[0], w).imag,
                                 np.vdot(w, w).real])
        d = np.array([raw[0] + 1j * raw[1]])
        start(0, d, raw[2])
        col, done = -1, False
        for K in range(1, stop_col + 1):  # pass K: update K-1, M A and projection of K
            U[K] = w - (d * vs[:K] ** 2) @ U[:K]
            passes += 1
            h_before = op.halo_calls
            w = ss[K] * op.psolve(op.apply(U[K]))  # (exchanges exactly u_K's edge rows)
            halos += op.halo_calls - h_before
            vals = sum(([c.real, c.imag] for c in (U[:K + 1].conj() @ w)), [])
            raw = counted_allreduce(vals + [np.vdot(w, w).real, np.vdot(U[K], U[K]).real])
            reduces += 1
            d = raw[0:2 * (K + 1):2] + 1j * raw[1:2 * (K + 1):2]
            sj = np.sqrt(raw[2 * (K + 1) + 1])
            vs[K] = 1 / sj
            col = K - 1
            if finish(col, sj * vs[K - 1] / ss[K - 1]):
                done = True
                break
            start(K, d, raw[2 * (K + 1)])
        if not done:  # the last update and its norm (one more reduction per cycle)
            U[stop_col + 1] = w - (d * vs[:stop_col + 1] ** 2) @ U[:stop_col + 1]
            sl = np.sqrt(counted_allreduce([np.vdot(U[stop_col + 1], U[stop_col + 1]).real])[0])
            col = stop_col
            vs[stop_col + 1] = 1 / sl
            finish(col, sl * vs[col] / ss[col])
        inner += col + 1
        if H[col, col] == 0:
            S[col] = 0
        y = S[:col + 1].copy()
        for k in range(col, 0, -1):
            if y[k] != 0:
                y[k] /= H[k, k]
                y[:k] -= y[k] * H[k, :k]
        if y[0] != 0:
            y[0] /= H[0, 0]
        x += (y * vs[:col + 1]) @ U[:col + 1]
        r = b - op.apply(x)
        rn = gnorm(r)
        per = max(passes, 1)
        if inner == maxiter:
            return x, (0 if rn <= atol else maxiter), np.array(hist), reduces / per, halos / per
        if rn <= atol or brk:
            break
        ptol_f = max(eps, 0.25 * ptol_f) if presid <= ptol else min(1.0, 1.5 * ptol_f)
        ptol = presid * min(ptol_f, atol / rn)
    per = max(passes, 1)
    return x, (0 if rn <= atol else maxiter), np.array(hist), reduces / per, halos / per
