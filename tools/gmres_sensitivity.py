"""How rounding-sensitive is the reference solve itself?  (CPU, oracle only.)

Runs scipy gmres exactly as code.py:516 calls it (oracle.gmres_reference) twice -- on f and
on f perturbed by 1e-15 relative -- and prints how far the presid history, the field and the
true residual drift apart.  Where the reference drifts by more than the 1e-6 contract, no
implementation can be held to it; DESIGN.md 6 uses this to choose the parity cases.
usage: python tools/gmres_sensitivity.py [n] [wave_num]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import helmholtz_oracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 600
wn = float(sys.argv[2]) if len(sys.argv) > 2 else 12.0
b, C, al = 12, 81.0, 2.0
cm = O.init_c1_mat(.5, .5, n)
om, h, eta = O.problem_params(n, b, wn, al)
A = O.build_A_matrix(b, C, eta, om, h, n, cm)
f = O.init_f1_mat(.5, .125, om, n).ravel()
fp = f * (1 + 1e-15 * np.random.default_rng(1).standard_normal(f.size))
precs = (("none", None), ("jacobi", O.jacobi_preconditioner(A)),
         ("sl", O.shifted_laplace_jacobi(b, C, eta, om, h, n, cm, beta=0.5, sweeps=2,
                                         damping=0.7)[0]))
print(f"n={n} wave_num={wn}: drift between scipy gmres on f and on f(1 + 1e-15 N(0,1))")
for name, M in precs:
    for x0s in (None, 1e-6):
        for K in (6, 12, 30):
            x0 = None if x0s is None else x0s * f
            x1, _, h1, r1 = O.gmres_reference(A, f, M=M, rtol=1e-3, restart=20, maxiter=K,
                                              x0=None if x0 is None else x0.copy())
            x2, _, h2, r2 = O.gmres_reference(A, fp, M=M, rtol=1e-3, restart=20, maxiter=K,
                                              x0=None if x0 is None else x0.copy())
            print(f"M={name:6s} x0={'0' if x0s is None else '1e-6 f':7s} iters={K:2d}: "
                  f"presid {np.max(np.abs(h1 - h2) / h1):.1e}  "
                  f"field {np.linalg.norm(x1 - x2) / np.linalg.norm(x1):.1e}  "
                  f"true relres {abs(r1 - r2) / r1:.1e}", flush=True)
