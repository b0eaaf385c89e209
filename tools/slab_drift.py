"""Where does the slab-split history drift come from?  

test_fused_pass_virtual_slabs_match_single_slab compares the one-pass GMRES on 1 slab with the
same solve on 2-4 virtual slabs of one rank.  Per point, u_K and w_K are formed by the same
arithmetic on either layout (a band's halo rows across a slab boundary are formed in place by
the same k-order update as the stored rows, FROW_MEM); what differs is the order in which the
projections' per-block partial rows add.  This tool measures, per inner iteration, the relative
history drift of:

  gpu-slabs   the device solve on 1 vs S virtual slabs (--gpu; the test's case)
  gpu-noise   the device solve on f vs f (1 + 1e-15 N(0,1)), 1 slab (--gpu)
  mirror      the numpy mirror of the runtime's one-pass order (tests/dist_mirror.py
              gmres_dist_onepass) over gloo, world 1 vs world S: the SAME algorithm, whose slab
              split changes nothing but the inner products' summation order (np.vdot per slab,
              then the allreduce)
  scipy-noise scipy gmres (the reference's solver) on f vs f (1 + 1e-15 N(0,1))

and the history itself (the drift is relative to presid, which falls by orders of magnitude).
usage: python tools/slab_drift.py [--n 613] [--slabs 4] [--precond jacobi] [--gpu]
"""
import argparse
import multiprocessing as mp
import os
import socket
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import helmholtz_oracle as O  # noqa: E402

WN, RTOL = 6.0, 1e-3
RESTART, ITERS = 12, 26  # the virtual-slab test's problem (--restart / --iters override)


def _mirror_worker(rank, world, port, n, precond, out, restart, iters):
    global RESTART, ITERS
    RESTART, ITERS = restart, iters
    import torch.distributed as dist
    import dist_mirror as DM
    from helmholtz_preconditioner_amd import dist as hdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    om, h, eta = O.problem_params(n, 12, WN, 2.0)
    j0, j1 = hdist.slab_bounds(n, world, rank)
    op = DM.SlabOperator(81.0, eta, om, h, n, O.init_c1_mat(.5, .5, n), j0, j1,
                         jacobi=precond == "jacobi")
    f = O.init_f1_mat(.5, .125, om, n)[j0:j1].ravel()
    x, info, hist, _, _ = DM.gmres_dist_onepass(op, f, RTOL, RESTART, ITERS)
    np.savez(out, x=x, hist=hist, j0=j0)
    dist.destroy_process_group()


def mirror(n, precond, world):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as td:
        outs = [os.path.join(td, f"r{r}.npz") for r in range(world)]
        ps = [ctx.Process(target=_mirror_worker, args=(r, world, port, n, precond, outs[r],
                                                       RESTART, ITERS))
              for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(timeout=600)
            assert p.exitcode == 0
        parts = [np.load(o) for o in outs]
        return parts[0]["hist"], np.concatenate([p["x"] for p in parts])


def scipy_noise(n, precond):
    om, h, eta = O.problem_params(n, 12, WN, 2.0)
    A = O.build_A_matrix(12, 81.0, eta, om, h, n, O.init_c1_mat(.5, .5, n))
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    fp = f * (1 + 1e-15 * np.random.default_rng(1).standard_normal(f.size))
    M = O.jacobi_preconditioner(A) if precond == "jacobi" else None
    x1, _, h1, _ = O.gmres_reference(A, f, M=M, rtol=RTOL, restart=RESTART, maxiter=ITERS)
    x2, _, h2, _ = O.gmres_reference(A, fp, M=M, rtol=RTOL, restart=RESTART, maxiter=ITERS)
    return h1, h2, x1, x2


def gpu(n, precond, slabs):
    import helmholtz_preconditioner_amd as H
    om, h, eta = H.problem_params(n, 12, WN, 2.0)
    cm = H.init_c1_mat(.5, .5, n)
    f = H.init_f1_mat(.5, .125, om, n).ravel()
    fp = f * (1 + 1e-15 * np.random.default_rng(1).standard_normal(f.size))
    out = {}
    for key, s, rhs in (("1", 1, f), ("S", slabs, f), ("noise", 1, fp)):
        c = H.Context(device=0, virtual_slabs=s)
        A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm, context=c)
        A.krylov_mode("fused")
        A.small_cycle("off")
        M = H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7) if precond == "sl" else precond
        _, _, hist = H.gmres(A, rhs, rtol=RTOL, restart=RESTART, maxiter=ITERS, M=M,
                             callback=lambda r: None, callback_type="legacy",
                             return_history=True)
        assert A.last_solve_path() == "one-pass"
        out[key] = np.asarray(hist)
        A.close()
        c.close()
    return out


def rel(a, b):
    m = min(len(a), len(b))
    return np.abs(a[:m] - b[:m]) / np.abs(a[:m])


def main():
    global RESTART, ITERS
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=613)
    p.add_argument("--slabs", type=int, default=4)
    p.add_argument("--precond", default="jacobi", choices=["none", "jacobi", "sl"])
    p.add_argument("--gpu", action="store_true")
    p.add_argument("--restart", type=int, default=RESTART)
    p.add_argument("--iters", type=int, default=ITERS)
    a = p.parse_args()
    RESTART, ITERS = a.restart, a.iters
    pc = None if a.precond == "none" else a.precond
    cols = {}
    if a.gpu:
        g = gpu(a.n, pc, a.slabs)
        cols[f"gpu 1 vs {a.slabs} slabs"] = rel(g["1"], g["S"])
        cols["gpu f vs f(1+1e-15)"] = rel(g["1"], g["noise"])
        hist = g["1"]
    if a.precond != "sl":  # (the mirror and the oracle restate none / Jacobi)
        (m1, mx1), (mS, mxS) = mirror(a.n, pc, 1), mirror(a.n, pc, a.slabs)
        cols[f"mirror world 1 vs {a.slabs}"] = rel(m1, mS)
        s1, s2, sx1, sx2 = scipy_noise(a.n, pc)
        cols["scipy f vs f(1+1e-15)"] = rel(s1, s2)
        fields = {f"mirror world 1 vs {a.slabs}": np.linalg.norm(mxS - mx1) / np.linalg.norm(mx1),
                  "scipy f vs f(1+1e-15)": np.linalg.norm(sx2 - sx1) / np.linalg.norm(sx1)}
        if not a.gpu:
            hist = s1
    print(f"n={a.n} c1 wave_num={WN} M={a.precond} GMRES({RESTART}) rtol={RTOL} "
          f"{ITERS} iterations: relative presid drift per inner iteration")
    print(f"{'it':>3s} {'presid':>10s} " + " ".join(f"{k:>24s}" for k in cols))
    for i in range(ITERS):
        row = [f"{cols[k][i]:24.2e}" if i < len(cols[k]) else f"{'-':>24s}" for k in cols]
        print(f"{i + 1:3d} {hist[i]:10.3e} " + " ".join(row))
    for k, v in cols.items():
        print(f"max over the first 10 / all iterations, {k}: {v[:10].max():.2e} / {v.max():.2e}")
    for k, v in (fields.items() if a.precond != "sl" else []):
        print(f"field relative difference after {ITERS} iterations, {k}: {v:.2e}")


if __name__ == "__main__":
    main()
