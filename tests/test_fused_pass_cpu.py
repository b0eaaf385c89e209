"""CPU tier: the decomposition the one-pass GMRES iteration (krylov.hip fused_iter_kernel,
DESIGN 3g) relies on, restated in numpy -- bands of rows that re-form their two halo rows of
u_{j+1}, strips whose edge columns are formed by the edge lanes -- gives the same update,
M A and projections as the three separate launches (update_kernel, stencil, multidot_kernel)
it replaces.  Host-side algebra only (no GPU); the kernel itself is checked against scipy and
the lagged path in tests/test_gpu_krylov_modes.py."""
import numpy as np
import pytest

from oracle import helmholtz_oracle as O


def _problem(n, seed):
    om, h, eta = O.problem_params(n, 6, 3.0, 2.0)
    A = O.build_A_matrix(6, 81.0, eta, om, h, n, O.init_c1_mat(.5, .5, n)).tocsr()
    rng = np.random.default_rng(seed)
    K = 5
    V = rng.standard_normal((K, n * n)) + 1j * rng.standard_normal((K, n * n))
    w = rng.standard_normal(n * n) + 1j * rng.standard_normal(n * n)
    coef = rng.standard_normal(K) + 1j * rng.standard_normal(K)
    return A, V, w, coef


def _separate(A, V, w, coef, s, jac):
    u = w - coef @ V                                      # update_kernel
    Au = A @ (s * u)
    wn = Au / A.diagonal() if jac else Au                 # stencil (+ Jacobi)
    Vn = np.vstack([V, u])
    return u, wn, np.conj(Vn) @ wn, np.vdot(wn, wn).real  # multidot_kernel


def _fused(A, V, w, coef, s, jac, n, R, S):
    """band height R, strip width S: every band forms u on its rows and its two halo rows,
    every strip on its columns and the two edge columns, from w and V only"""
    u_out = np.zeros(n * n, complex)
    w_out = np.zeros(n * n, complex)
    dots = np.zeros(V.shape[0] + 1, complex)
    nw = 0.0
    d = A.diagonal()
    for rb in range(0, n, R):
        re = min(rb + R, n)
        for i0 in range(0, n, S):
            i1 = min(i0 + S, n)
            rows = range(rb - 1, re + 1)
            cols = range(i0 - 1, i1 + 1)
            loc = {}
            for r in rows:                    # u_K on the band + halo rows, strip + edges
                for c in cols:
                    if 0 <= r < n and 0 <= c < n:
                        p = r * n + c
                        loc[(r, c)] = w[p] - coef @ V[:, p]
            for r in range(rb, re):
                for c in range(i0, i1):
                    p = r * n + c
                    row = A.getrow(p)
                    Au = sum(a * s * loc[(q // n, q % n)] for q, a in zip(row.indices, row.data))
                    wp = Au / d[p] if jac else Au
                    u_out[p] = loc[(r, c)]
                    w_out[p] = wp
                    dots += np.conj(np.append(V[:, p], loc[(r, c)])) * wp
                    nw += abs(wp) ** 2
    return u_out, w_out, dots, nw


@pytest.mark.parametrize("n,R,S,jac", [(13, 4, 8, True), (16, 8, 16, False), (11, 3, 5, True)])
def test_band_strip_decomposition_matches_separate_launches(n, R, S, jac):
    A, V, w, coef = _problem(n, n)
    s = 0.37
    u1, w1, d1, n1 = _separate(A, V, w, coef, s, jac)
    u2, w2, d2, n2 = _fused(A, V, w, coef, s, jac, n, R, S)
    assert np.allclose(u2, u1, rtol=0, atol=1e-12 * np.abs(u1).max())
    assert np.allclose(w2, w1, rtol=0, atol=1e-12 * np.abs(w1).max())
    assert np.allclose(d2, d1, rtol=1e-12)
    assert abs(n2 - n1) <= 1e-12 * n1
