"""One rank of a multi-process row-slab run (used by tests/test_gpu_dist.py).

Every rank runs on device 0, so the N > 1 orchestration (slab ownership, halo exchange,
global reductions inside GMRES, the preconditioners) is exercised on a single GPU, over
  * --transport shm: the host-staged shared-memory transport (csrc/comm.cpp ShmComm), or
  * --transport rccl: the production RcclComm itself.  RCCL refuses two ranks on one GPU
    of one host, so the parent gives every rank its own NCCL_HOSTID (RCCL then sees one
    rank per "host" and connects them through its socket transport over loopback): the
    communicator init, grouped halo send/recv on the priority stream, the allreduces and
    their ordering against the stencil launches all run as in production, only the wire
    between the ranks differs from xGMI.
Results go to an .npz for the parent.
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
    p.add_argument("--n", type=int, default=150)
    p.add_argument("--slabs", type=int, default=1)
    p.add_argument("--stencil", type=int, default=5)
    p.add_argument("--apply-only", action="store_true")
    p.add_argument("--transport", default="shm", choices=["shm", "rccl"])
    p.add_argument("--krylov", default="auto", help="krylov mode of the solves (auto, one, fused)")
    p.add_argument("--default-limits", action="store_true",
                   help="also solve with scipy's default restart / maxiter (global-N based)")
    a = p.parse_args()
    if a.transport == "rccl":
        from helmholtz_preconditioner_amd import dist
        uid = dist.exchange_unique_id(a.rank, a.world, key=a.id[:32], timeout=120.0)
    else:
        uid = bytes.fromhex(a.id)
    ctx = H.Context(device=0, rank=a.rank, world=a.world, nccl_id=uid,
                    virtual_slabs=a.slabs, transport=a.transport)
    if a.transport == "rccl":
        ctx.barrier()
        if a.rank == 0:
            dist.cleanup_rendezvous(a.id[:32])
    n = a.n
    om, h, eta = H.problem_params(n, 12, 6.0, 2.0)
    cm = H.init_c1_mat(.5, .5, n)
    A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm, context=ctx, stencil=a.stencil)
    A.krylov_mode(a.krylov)
    j0, j1 = A.row_begin, A.row_end
    rng = np.random.default_rng(5)
    xg = (rng.standard_normal(n * n) + 1j * rng.standard_normal(n * n)).reshape(n, n)
    y = A @ xg[j0:j1].ravel()
    f = H.init_f1_mat(.5, .125, om, n)[j0:j1].ravel()
    out = dict(j0=j0, j1=j1, y=y)
    # the two-sweep shifted-Laplace M A (fused: two halo rows exchanged across ranks)
    Msl = H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7)
    Msl.configure()
    out["ysl"] = A._apply_host(xg[j0:j1].ravel(), H._ffi.HH_APPLY_PREC_A)
    for name, M in () if a.apply_only else (("none", None), ("jacobi", "jacobi"),
                    ("sl", H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7))):
        x, info, hist = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=50, M=M,
                                callback=lambda r: None, callback_type="legacy",
                                return_history=True)
        out[f"x_{name}"], out[f"info_{name}"], out[f"hist_{name}"] = x, info, hist
        out[f"path_{name}"] = A.last_solve_path()
    if a.default_limits:
        x, info = H.gmres(A, f, rtol=1e-3, M="jacobi")
        out["x_default"], out["info_default"] = x, info
    # a host collective the bench uses for its timing
    out["maxrank"] = ctx.allreduce_max([float(a.rank)])[0]
    np.savez(a.out, **out)
    ctx.barrier()


if __name__ == "__main__":
    main()
