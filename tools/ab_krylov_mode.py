"""A/B of the GMRES inner-iteration modes on one grid, interleaved in one process: "two"
(projections, then the updated vector's norm), "one" (lagged normalisation, one reduction
per iteration) and "fused" (one pass over the basis per iteration; env MODES selects), BASELINE config 2 by default (1024^2, constant medium, wn 64, Jacobi,
GMRES(20), K = 100 inner iterations).  usage: python tools/ab_krylov_mode.py [n] [wn] [reps]
env VSLABS=S: the grid as S virtual slabs of one rank (one pass launch per slab: the per-rank
slab shapes of an S-rank run, for PMC records of N > 1 lines)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import helmholtz_preconditioner_amd as H  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
wn = float(sys.argv[2]) if len(sys.argv) > 2 else 64.0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
K = 100
MODES = [m for m in os.environ.get("MODES", "two,one,fused").split(",")]
om, h, eta = H.problem_params(n, 12, wn, 2.0)
PRE = os.environ.get("PRECOND", "jacobi")  # jacobi | sl (config 3: Marmousi-like, SL beta 0.5)
cm = H.marmousi_like_c_mat(n) if PRE == "sl" else H.constant_c_mat(n)
VS = int(os.environ.get("VSLABS", "1"))
ctx = H.Context(device=0, virtual_slabs=VS) if VS > 1 else None
A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm, context=ctx)
f = H.init_f1_mat(.5, .125, om, n).ravel()
M = H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7) if PRE == "sl" else "jacobi"
hist = {}
for r in range(reps + 1):
    for mode in MODES:
        A.krylov_mode(mode)
        t0 = time.perf_counter()
        u, info, hh = H.gmres(A, f, rtol=1e-12, restart=20, maxiter=K, M=M,
                              callback=lambda x: None, callback_type="legacy",
                              return_history=True)
        dt = time.perf_counter() - t0
        hist[mode] = (u, np.asarray(hh))
        if r > 0:
            print(f"n={n} mode={mode}: {len(hh) / dt:9.1f} it/s", flush=True)
u2, h2 = hist[MODES[0]]
for m in MODES[1:]:
    u1, h1 = hist[m]
    print(f"{m} vs {MODES[0]}: history max rel diff {np.max(np.abs(h1 - h2) / h2):.2e}, "
          f"field rel diff {np.linalg.norm(u1 - u2) / np.linalg.norm(u2):.2e}")
