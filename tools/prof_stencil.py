"""Profiling driver: only the operator apply (and optionally one GMRES cycle) at the bench
workload, so rocprofv3 kernel-trace / PMC passes stay short.
usage: python tools/prof_stencil.py [--n 4096] [--iters 50] [--medium marmousi] [--gmres]
                                   [--stencil 9]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import helmholtz_preconditioner_amd as H  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=4096)
p.add_argument("--iters", type=int, default=50)
p.add_argument("--medium", default="marmousi")
p.add_argument("--gmres", action="store_true")
p.add_argument("--variant", type=int, default=-1)
p.add_argument("--rpb", type=int, default=0)
p.add_argument("--rotate", type=int, default=3, help="distinct (x, y) pairs, as bench.py")
p.add_argument("--stencil", type=int, default=5, choices=[5, 9])
p.add_argument("--virtual-slabs", type=int, default=1,
               help="the grid as S slabs of one rank: one apply launch per slab (a rank's slab "
                    "shape of an S-rank run)")
a = p.parse_args()
n = a.n
om, h, eta = H.problem_params(n, 12, 100.0, 2.0)
cm = H.marmousi_like_c_mat(n) if a.medium == "marmousi" else H.constant_c_mat(n)
ctx = H.Context(device=0, virtual_slabs=a.virtual_slabs) if a.virtual_slabs > 1 else None
A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm, stencil=a.stencil, context=ctx)
if a.variant >= 0 or a.rpb > 0:
    A.tune(variant=a.variant, rows_per_block=a.rpb)
xs, ys = [A.vector() for _ in range(a.rotate)], [A.vector() for _ in range(a.rotate)]
for j, v in enumerate(xs):
    v.fill_hash(7 + j)
tot, k = A.time_apply(xs, ys, a.iters)
bpp = A.bytes_per_point
print(f"n={n} iters={a.iters} kernel {k*1e3:.1f} us  {bpp*n*n/(k*1e-3)/1e9:.0f} GB/s  total/iter {tot/a.iters*1e3:.1f} us")
if a.gmres:
    f = A.vector(H.init_f1_mat(.5, .125, om, n).ravel())
    H.gmres(A, f, rtol=1e-14, restart=20, maxiter=20, M=H.ShiftedLaplace(A, 0.5, 2, 0.7),
            callback=lambda r: None, callback_type="legacy")
