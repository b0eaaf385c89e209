"""CPU tier: the partitioned block-Thomas solve's carry algebra (sweep.hip
bt_solve_chunked), restated in numpy and checked against the sequential recurrence it replaces
-- the affine recurrences y_i = c_i + M_i y_{i-1} (forward) and x_i = y_i + N_i x_{i+1}
(backward) of a block-Thomas solve (reference code.py:229-291, the sweeps' H_m solves), cut
into G workgroups of 16 chunks: chunk-local zero-carry runs, the 16-step chunk chain, the
product-form grid step (grid maps T(w, u) = Phi_{w-1} .. Phi_{u+1}, identity for the nearest
upstream workgroup, sweep_grid_setup_kernel) and the per-chunk carry through the workgroup
prefix maps Pw.  Random well-conditioned blocks stand in for the factors (the algebra is the
same for any maps); the GPU tier checks the kernels against the sequential solves and the
oracle (tests/test_gpu_sweep.py)."""
import numpy as np
import pytest

KL = 16  # chunks per workgroup (kSweepChunks)


def chunk_lo(n, K, k):
    return n * k // K


def sequential(M, c):
    y, out = np.zeros(M[0].shape[0], complex), []
    for Mi, ci in zip(M, c):
        y = ci + Mi @ y
        out.append(y)
    return np.array(out)


def partitioned(M, c, G):
    """The forward recurrence as the partitioned solve computes it (the backward one is the
    same algebra on reversed columns)."""
    n, B = len(M), M[0].shape[0]
    K = KL * G
    I = np.eye(B)
    # chunk-local zero-carry runs and chunk maps F (Psi at the chunk's last column)
    yl, F = [], []
    for k in range(K):
        y, P = np.zeros(B, complex), I.copy()
        for i in range(chunk_lo(n, K, k), chunk_lo(n, K, k + 1)):
            y, P = c[i] + M[i] @ y, M[i] @ P
        yl.append(y)
        F.append(P)
    # per workgroup: the 16-step zero-carry chain, its published end vector e, prefix maps Pw
    z, e, Pw, Phi = [], [], [], []
    for w in range(G):
        zw, v, pw, P = [], np.zeros(B, complex), [], I.copy()
        for q in range(KL):
            k = KL * w + q
            v = yl[k] + F[k] @ v
            P = F[k] @ P
            zw.append(v)
            pw.append(P.copy())
        z.append(zw)
        e.append(v)
        Pw.append(pw)
        Phi.append(P)
    # grid maps T(w, u) for distances >= 2, built like sweep_grid_setup_kernel (left products
    # walking the downstream workgroups of each upstream one)
    T = {}
    for u in range(G):
        P = None
        for wd in range(u + 2, G):
            P = Phi[wd - 1] if P is None else Phi[wd - 1] @ P
            T[(wd, u)] = P
    # the grid step: carry_in(w) = sum_u T(w, u) e_u, identity for u = w - 1
    carry = [np.zeros(B, complex)]
    for w in range(1, G):
        acc = e[w - 1].copy()
        for u in range(w - 1):
            acc = acc + T[(w, u)] @ e[u]
        carry.append(acc)
    # fix-up: each chunk's true carry in ONE step, then its columns
    y = np.zeros((n, B), complex)
    for w in range(G):
        for q in range(KL):
            k = KL * w + q
            cin = carry[w] if q == 0 else z[w][q - 1] + Pw[w][q - 1] @ carry[w]
            v = cin
            for i in range(chunk_lo(n, K, k), chunk_lo(n, K, k + 1)):
                v = c[i] + M[i] @ v
                y[i] = v
    return y


@pytest.mark.parametrize("n,B,G", [(64, 4, 1), (96, 4, 3), (200, 8, 5), (333, 4, 10),
                                   (1100, 4, 34)])
def test_partitioned_carries_match_the_sequential_recurrence(n, B, G):
    rng = np.random.default_rng(n + B + G)
    M = [0.45 * (rng.standard_normal((B, B)) + 1j * rng.standard_normal((B, B))) / np.sqrt(B)
         for _ in range(n)]
    c = [rng.standard_normal(B) + 1j * rng.standard_normal(B) for _ in range(n)]
    ys = sequential(M, c)
    yp = partitioned(M, c, G)
    assert np.linalg.norm(yp - ys) <= 1e-12 * np.linalg.norm(ys)


def test_grid_map_indexing_matches_the_device_layout():
    """sweep_grid_tri (sweep.hpp): workgroup w with cnt upstream workgroups keeps its maps for
    distances 2 .. cnt at tri(cnt) + d - 2, tri(cnt) = (cnt - 1)(cnt - 2) / 2 -- a dense,
    non-overlapping triangle of (G - 1)(G - 2) / 2 maps per system and direction"""
    tri = lambda cnt: (cnt - 1) * (cnt - 2) // 2 if cnt >= 2 else 0  # noqa: E731
    for G in (1, 2, 3, 17, 64):
        slots = [tri(cnt) + d - 2 for cnt in range(G) for d in range(2, cnt + 1)]
        assert sorted(slots) == list(range(tri(G)))
