"""Sweep stencil variants x band heights at the bench workload, interleaved rounds in one
process (methodology: cdna_hip_programming.md 5.4 rule 24), and check every variant's
output is bit-identical to variant 0 on a ragged grid.
usage: python tools/tune_stencil.py [--n 4096] [--rounds 3] [--iters 50]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import helmholtz_preconditioner_amd as H  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=4096)
p.add_argument("--rounds", type=int, default=3)
p.add_argument("--iters", type=int, default=50)
p.add_argument("--variants", default="6,7,9,24,30,31,33")
p.add_argument("--grids", default="0,1280")
p.add_argument("--rpbs", default="16,32,64")
p.add_argument("--medium", default="marmousi")
p.add_argument("--rotate", type=int, default=1,
               help="distinct (x, y) pairs applied round-robin (>1: no cross-launch cache reuse)")
a = p.parse_args()
variants = [int(v) for v in a.variants.replace("/", ",").split(",")]  # (/: gpu_session.sh args)
rpbs = [int(v) for v in a.rpbs.replace("/", ",").split(",")]
grids = [int(v) for v in a.grids.replace("/", ",").split(",")]


def vname(v):
    if v >= 96:  # non-marching tiles (stencil.hip kTileVariant ...)
        w = v - 96
        kind = {0: "tile", 1: "tile ntu", 2: "tile st-cached", 3: "tile st-cached", 4: "tile persist",
                6: "tile privnt"}.get(w // 16, "tile ?")
        return f"{kind} R{w % 16}"
    w = v % 24
    return f"{['lds', 'direct', 'shfl'][w % 3]} pf{(w // 3) % 2 + 1}{' nt' if (w // 6) % 2 else ''}" \
           f"{' ntu' if w >= 12 else ''}{' w512' if v % 48 >= 24 else ''}{' occ6' if v >= 48 else ''}"

# correctness on a ragged grid: every variant bit-identical to variant 0
n = 1000
om, h, eta = H.problem_params(n, 12, 30.0, 2.0)
A = H.build_A_matrix(12, 81.0, eta, om, h, n, H.marmousi_like_c_mat(n))
x, y = A.vector(), A.vector()
x.fill_hash(3)
A.tune(0, 0, 0)
A.apply_device(x, y)
ref = y.download()
for v in variants:
    for r, g in ((0, 0), (8, 0), (0, 64), (8, 24)):
        A.tune(v, r, g)
        A.apply_device(x, y)
        d = y.download()
        assert np.array_equal(d, ref), (v, r, np.abs(d - ref).max())
print("all variants bit-identical on n=1000", flush=True)
del A, x, y

n = a.n
om, h, eta = H.problem_params(n, 12, 100.0, 2.0)
cm = H.marmousi_like_c_mat(n) if a.medium == "marmousi" else H.constant_c_mat(n)
A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm)
xs, ys = [A.vector() for _ in range(a.rotate)], [A.vector() for _ in range(a.rotate)]
for k, v in enumerate(xs):
    v.fill_hash(7 + k)
x, y = (xs, ys) if a.rotate > 1 else (xs[0], ys[0])
bpp = A.bytes_per_point
res = {}
for rnd in range(a.rounds):
    for v in variants:
        for r in rpbs:
            for g in grids:
                A.tune(v, r, g)
                A.time_apply(x, y, 5)
                tot, k = A.time_apply(x, y, a.iters)
                res.setdefault((v, r, g), []).append(k)
rows = []
for (v, r, g), ks in res.items():
    k = min(ks)
    rows.append((bpp * n * n / (k * 1e-3) / 1e9, v, r, g, k, np.median(ks)))
rows.sort(reverse=True)
import ctypes
from helmholtz_preconditioner_amd import _ffi
if not A.constant_medium:
    km = ctypes.c_double()
    ks = []
    for _ in range(a.rounds):
        _ffi.check(_ffi.lib.hh_op_probe_stream(A.handle, 0, 8192, xs[0].handle, ys[0].handle, a.iters, ctypes.byref(km), ctypes.byref(ctypes.c_int())))
        ks.append(km.value)
    k = min(ks)
    print(f"probe y=u*ic (same 40 B/pt, no neighbours): {k*1e3:.1f} us = {bpp*n*n/(k*1e-3)/1e9:.0f} GB/s")
print(f"n={n} medium={a.medium} bytes/pt={bpp} rotate={a.rotate}")
print("GB/s(best)  variant               rpb  grid  kernel_us(min)  kernel_us(median)")
for gbs, v, r, g, k, med in rows:
    desc = f"{v:2d} {vname(v)}"
    print(f"{gbs:9.0f}   {desc:20s} {r:4d} {g:5d}   {k * 1e3:9.1f}   {med * 1e3:9.1f}")
