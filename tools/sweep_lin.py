"""Linearity and workgroup-count agreement of the partitioned sweep (diagnostic):
python tools/sweep_lin.py N WGS [WGS ...] -- per G: relerr(M(x + 2i y), M x + 2i M y) and
relerr(M_G x, M_G0 x) against the first G."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import helmholtz_preconditioner_amd as H  # noqa: E402

n = int(sys.argv[1])
wgs = [int(v) for v in sys.argv[2:]] or [0]
b = 12
om, h, eta = H.problem_params(n, b, 100.0, 2.0)
cm, _ = H.init_c1_f1(om, n)
A = H.build_A_matrix(b, 81.0, eta, om, h, n, cm)
rng = np.random.default_rng(1)
x = rng.standard_normal(n * n) + 1j * rng.standard_normal(n * n)
y = rng.standard_normal(n * n) + 1j * rng.standard_normal(n * n)
rel = lambda a, c: float(np.linalg.norm(a - c) / np.linalg.norm(c))  # noqa: E731
ref = None
for g in wgs:
    M = H.Sweeping(A, form="thomas", workgroups=g)
    M.configure()
    mx, my, mxy = M @ x, M @ y, M @ (x + 2j * y)
    mx2 = M @ x
    ref = mx if ref is None else ref
    print(f"n={n} G={M.workgroups}: linearity {rel(mxy, mx + 2j * my):.2e}  repeat "
          f"{rel(mx2, mx):.2e}  vs first {rel(mx, ref):.2e}", flush=True)
    del M
