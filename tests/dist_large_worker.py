"""One rank of a BASELINE config-4 / config-5 run (8192^2 / 16384^2 constant medium, used by
tests/test_gpu_configs.py): every rank sits on device 0, over the shared-memory transport or
the production RCCL one (--transport; RCCL then needs one NCCL host id per rank, which the
parent sets in the environment).

The input is the hash fill (hh_vec_fill_hash: a pure function of the global index, identical
for any slab decomposition), so nothing of size N crosses the process boundary on the way in;
the parent's single-domain results are memory-mapped from .npy files and compared here, rank
by rank, and only small summaries come back.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import helmholtz_preconditioner_amd as H  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rank", type=int)
    p.add_argument("--world", type=int)
    p.add_argument("--id")
    p.add_argument("--out")
    p.add_argument("--n", type=int)
    p.add_argument("--wave-num", type=float)
    p.add_argument("--iters", type=int)
    p.add_argument("--ref-dir")
    p.add_argument("--transport", default="shm", choices=["shm", "rccl"])
    p.add_argument("--no-apply", action="store_true", help="skip the apply comparison")
    a = p.parse_args()
    if a.transport == "rccl":  # rank 0's ncclGetUniqueId, shipped through a node-local file
        from helmholtz_preconditioner_amd import dist
        uid = dist.exchange_unique_id(a.rank, a.world, key=a.id[:32], timeout=120.0)
    else:
        uid = bytes.fromhex(a.id)
    ctx = H.Context(device=0, rank=a.rank, world=a.world, nccl_id=uid, transport=a.transport)
    if a.transport == "rccl":
        ctx.barrier()
        if a.rank == 0:
            dist.cleanup_rendezvous(a.id[:32])
    n = a.n
    om, h, eta = H.problem_params(n, 12, a.wave_num, 2.0)
    A = H.build_A_matrix(12, 81.0, eta, om, h, n, np.broadcast_to(1.0, (n + 2, n + 2)),
                         context=ctx)
    j0, j1 = A.row_begin, A.row_end
    out = dict(j0=j0, j1=j1, transport=a.transport, y_mismatch=-1)
    if not a.no_apply:
        x, y = A.vector(), A.vector()
        x.fill_hash(7)
        A.apply_device(x, y)
        yl = y.download()
        x.close()
        y.close()
        yref = np.load(os.path.join(a.ref_dir, "y.npy"), mmap_mode="r")[j0 * n:j1 * n]
        out["y_mismatch"] = int(np.count_nonzero(yl != yref))
        del yl, yref
    f = H.init_f1_rows(.5, .125, om, n, j0, j1).ravel()  # (rows j0 .. j1 of init_f1_mat)
    xs, info, hist = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=a.iters, M="jacobi",
                             callback=lambda r: None, callback_type="legacy",
                             return_history=True)
    xref = np.load(os.path.join(a.ref_dir, "x.npy"), mmap_mode="r")[j0 * n:j1 * n]
    out.update(info=info, hist=hist, dx2=float(np.sum(np.abs(xs - xref) ** 2)),
               x2=float(np.sum(np.abs(xref) ** 2)), path=A.last_solve_path())
    np.savez(a.out, **out)
    ctx.barrier()


if __name__ == "__main__":
    main()
