"""Shapes of the fused shifted-Laplace M A kernel (csrc/sl_fused.hip) at the bench workload:
strip width (256 / 512) x NT or cached v loads x band height, cold inputs (3 rotating pairs),
interleaved rounds; every shape bit-identical (checked).
usage: python tools/tune_sl2.py [--n 4096] [--rounds 2] [--iters 40]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import helmholtz_preconditioner_amd as H  # noqa: E402
from helmholtz_preconditioner_amd import _ffi  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=4096)
p.add_argument("--rounds", type=int, default=2)
p.add_argument("--iters", type=int, default=40)
p.add_argument("--rpbs", default="8,16,32,64")
p.add_argument("--variants", default="6,18,30,42")
p.add_argument("--stencil", type=int, default=5, choices=[5, 9])
a = p.parse_args()
n = a.n
om, h, eta = H.problem_params(n, 12, 100.0, 2.0)
A = H.build_A_matrix(12, 81.0, eta, om, h, n, H.marmousi_like_c_mat(n), stencil=a.stencil)
A.set_preconditioner(_ffi.HH_PREC_SHIFTED_LAPLACE, 0.5, 2, 0.7)
xs = [A.vector() for _ in range(3)]
ys = [A.vector() for _ in range(3)]
for k, v in enumerate(xs):
    v.fill_hash(3 + k)
shapes = [(v, r) for v in [int(t) for t in a.variants.split(",")]
          for r in [int(t) for t in a.rpbs.split(",")]]
ref = None
for v, r in shapes:
    A.tune(v, r)
    A.apply_device(xs[0], ys[0], _ffi.HH_APPLY_PREC_A)
    out = ys[0].download()
    ref = out if ref is None else ref
    assert np.array_equal(out, ref), (v, r)
print(f"all fused M A shapes bit-identical at n={n}")
best = {}
for rnd in range(a.rounds):
    for v, r in shapes + [(-1, 0)]:
        A.tune(v, r)
        t, _ = A.time_apply(xs, ys, a.iters, _ffi.HH_APPLY_PREC_A)
        best[(v, r)] = min(best.get((v, r), 1e9), t / a.iters)
print(f"n={n} marmousi, M A (2 sweeps), 40 B/unknown, cold inputs (3 pairs)")
print("variant  rpb   us/apply  GB/s   (variant -1 rpb 0 = built-in default)")
for (v, r), t in sorted(best.items(), key=lambda q: q[1]):
    print(f"{v:7d}  {r:3d}  {t * 1e3:9.1f}  {40 * n * n / (t * 1e-3) / 1e9:5.0f}")
