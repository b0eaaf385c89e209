"""A/B the Krylov streaming kernels in one process: NT basis loads x grid size, timing a
fixed number of GMRES(20) inner iterations at the bench workload (interleaved rounds)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import helmholtz_preconditioner_amd as H  # noqa: E402
from helmholtz_preconditioner_amd import _ffi  # noqa: E402

# usage: tune_krylov.py [n [config]]  -- config 3 (default): Marmousi-like, shifted-Laplace,
# wn 100; config 2: constant medium, Jacobi, wn 64 (BASELINE.json)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
config = int(sys.argv[2]) if len(sys.argv) > 2 else 3
om, h, eta = H.problem_params(n, 12, 100.0 if config == 3 else 64.0, 2.0)
cm = H.marmousi_like_c_mat(n) if config == 3 else np.ones((n + 2, n + 2))
A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm)
f = A.vector(H.init_f1_mat(.5, .125, om, n).ravel())
M = H.ShiftedLaplace(A, 0.5, 2, 0.7) if config == 3 else "jacobi"
grid = (1024, 2048, 4096, 8192) if n >= 2048 else (256, 512, 768, 1024, 2048, 4096)
res = {}
for rnd in range(3):
    for nt in (0, 1):
        for blocks in grid:
            _ffi.check(_ffi.lib.hh_tune_krylov(nt, blocks))
            H.gmres(A, f, rtol=1e-14, restart=20, maxiter=2, M=M, callback=lambda r: None,
                    callback_type="legacy")
            A.ctx.synchronize()
            t0 = time.perf_counter()
            H.gmres(A, f, rtol=1e-14, restart=20, maxiter=40, M=M, callback=lambda r: None,
                    callback_type="legacy")
            res.setdefault((nt, blocks), []).append(time.perf_counter() - t0)
for (nt, blocks), ts in sorted(res.items(), key=lambda kv: min(kv[1])):
    print(f"nt={nt} blocks={blocks:5d}  {40 / min(ts):7.1f} it/s (best)  {40 / np.median(ts):7.1f} (median)")
