"""9-point stencil shapes at the bench workload: the three strip shapes the
9-point operator instantiates x band heights, cold inputs (rotating vector pairs), interleaved
rounds in one process, next to the 5-point default.  Every shape is bit-identical (checked).
usage: python tools/tune_stencil9.py [--n 4096] [--rounds 2] [--iters 50]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import helmholtz_preconditioner_amd as H  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=4096)
p.add_argument("--rounds", type=int, default=2)
p.add_argument("--iters", type=int, default=50)
p.add_argument("--rpbs", default="16,32,64")
p.add_argument("--medium", default="marmousi")
p.add_argument("--variants", default="")
a = p.parse_args()
n = a.n
om, h, eta = H.problem_params(n, 12, 100.0, 2.0)
cm = H.marmousi_like_c_mat(n) if a.medium == "marmousi" else H.constant_c_mat(n)
A9 = H.build_A_matrix(12, 81.0, eta, om, h, n, cm, stencil=9)
A5 = H.build_A_matrix(12, 81.0, eta, om, h, n, cm)
xs = [A9.vector() for _ in range(3)]
ys = [A9.vector() for _ in range(3)]
x5 = [A5.vector() for _ in range(3)]
y5 = [A5.vector() for _ in range(3)]
for k, v in enumerate(xs):
    v.fill_hash(7 + k)
    x5[k].fill_hash(7 + k)
bpp = A9.bytes_per_point
ref = None
shapes = [(v, r) for v in ([int(t) for t in a.variants.split(",")] if a.variants else (6, 18, 30, 42)) for r in [int(t) for t in a.rpbs.split(",")]]
for v, r in shapes:
    A9.tune(v, r)
    A9.apply_device(xs[0], ys[0])
    out = ys[0].download()
    if ref is None:
        ref = out
    assert np.array_equal(out, ref), (v, r)
print(f"all 9-point shapes bit-identical at n={n}")
best = {}
for rnd in range(a.rounds):
    for v, r in shapes + [("5pt", 0)]:
        if v == "5pt":
            A5.tune(-1, 0)
            _, k = A5.time_apply(x5, y5, a.iters)
        else:
            A9.tune(v, r)
            _, k = A9.time_apply(xs, ys, a.iters)
        best[(v, r)] = min(best.get((v, r), 1e9), k)
print(f"n={n} medium={a.medium} bytes/pt={bpp} cold inputs (3 pairs)")
print("shape                 rpb   kernel_us(min)  GB/s")
for (v, r), k in sorted(best.items(), key=lambda t: t[1]):
    print(f"{str(v):20s}  {r:4d}  {k * 1e3:12.1f}  {bpp * n * n / (k * 1e-3) / 1e9:7.0f}")
