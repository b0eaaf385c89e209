"""Diagnostic: repeatability of the row-slab path (tests/test_gpu_dist.py's flaky case).

Single process (world 1): GMRES 'none' / 'jacobi' / 'sl' R times, histories compared bitwise.
Multi-process (SHM transport, W ranks x S slabs on device 0): R device applies of one vector
compared bitwise with the first, then GMRES 'none' R times compared bitwise; each rank
prints its own verdict.
usage: python tools/stress_dist.py single|multi [W S R]
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import helmholtz_preconditioner_amd as H  # noqa: E402

N = 150


def problem(ctx):
    om, h, eta = H.problem_params(N, 12, 6.0, 2.0)
    A = H.build_A_matrix(12, 81.0, eta, om, h, N, H.init_c1_mat(.5, .5, N), context=ctx)
    f = H.init_f1_mat(.5, .125, om, N)[A.row_begin:A.row_end].ravel()
    return A, f


def gmres_hist(A, f, M):
    x, info, hist = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=50, M=M,
                            callback=lambda r: None, callback_type="legacy", return_history=True)
    return hist, x


def single(R):
    ctx = H.Context(device=0)
    A, f = problem(ctx)
    for name, M in (("none", None), ("jacobi", "jacobi"),
                    ("sl", H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7))):
        h0, x0 = gmres_hist(A, f, M)
        bad = 0
        for r in range(R):
            h, x = gmres_hist(A, f, M)
            if not (np.array_equal(h, h0) and np.array_equal(x, x0)):
                bad += 1
                k = int(np.argmax(h != h0)) if len(h) == len(h0) else -1
                print(f"single {name} run {r}: differs (first iteration {k}, "
                      f"max rel {np.max(np.abs(h - h0) / h0) if len(h) == len(h0) else 'len'})")
        print(f"single {name}: {bad}/{R} runs differ", flush=True)


def worker(rank, world, tok, slabs, R):
    ctx = H.Context(device=0, rank=rank, world=world, nccl_id=bytes.fromhex(tok),
                    virtual_slabs=slabs, transport="shm")
    A, f = problem(ctx)
    x = A.vector()
    x.fill_hash(7)
    y0, y = A.vector(), A.vector()
    A.apply_device(x, y0)
    ref = y0.download()
    bad = 0
    for r in range(R * 20):
        A.apply_device(x, y)
        if not np.array_equal(y.download(), ref):
            bad += 1
    print(f"rank {rank}: apply {bad}/{R * 20} differ", flush=True)
    h0, x0 = gmres_hist(A, f, None)
    badg = 0
    for r in range(R):
        h, xx = gmres_hist(A, f, None)
        if not (np.array_equal(h, h0) and np.array_equal(xx, x0)):
            badg += 1
            k = int(np.argmax(h != h0)) if len(h) == len(h0) else -1
            print(f"rank {rank} gmres run {r}: differs from iteration {k}", flush=True)
    print(f"rank {rank}: gmres none {badg}/{R} runs differ", flush=True)
    ctx.barrier()


def multi(W, S, R):
    tok = os.urandom(128).hex()
    procs = [subprocess.Popen([sys.executable, __file__, "worker", str(r), str(W), tok, str(S), str(R)])
             for r in range(W)]
    rc = [p.wait(timeout=600) for p in procs]
    print("multi rcs", rc, flush=True)
    return max(abs(c) for c in rc)


if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "single":
        single(int(sys.argv[2]) if len(sys.argv) > 2 else 5)
    elif mode == "multi":
        W, S, R = (int(v) for v in sys.argv[2:5])
        sys.exit(multi(W, S, R))
    else:
        worker(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5]), int(sys.argv[6]))
