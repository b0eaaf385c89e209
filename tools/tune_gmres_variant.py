"""A/B stencil variants inside the GMRES loop (every epilogue follows A.tune): timed GMRES(20)
inner iterations at the bench workload, interleaved rounds in one process.
usage: python tools/tune_gmres_variant.py [n] [variants, default 42,30]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import helmholtz_preconditioner_amd as H  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
variants = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "42,30").split(",")]
om, h, eta = H.problem_params(n, 12, 100.0, 2.0)
A = H.build_A_matrix(12, 81.0, eta, om, h, n, H.marmousi_like_c_mat(n))
f = A.vector(H.init_f1_mat(.5, .125, om, n).ravel())
res = {}
for pc in ("sl", "jacobi", "none"):
    M = {"sl": lambda: H.ShiftedLaplace(A, 0.5, 2, 0.7), "jacobi": lambda: H.Jacobi(A),
         "none": lambda: None}[pc]()
    for rnd in range(3):
        for v in variants:
            A.tune(v, 0, 0)
            H.gmres(A, f, rtol=1e-14, restart=20, maxiter=2, M=M, callback=lambda r: None,
                    callback_type="legacy")
            A.ctx.synchronize()
            t0 = time.perf_counter()
            H.gmres(A, f, rtol=1e-14, restart=20, maxiter=40, M=M, callback=lambda r: None,
                    callback_type="legacy")
            res.setdefault((pc, v), []).append(time.perf_counter() - t0)
for (pc, v), ts in sorted(res.items()):
    print(f"precond={pc:6s} variant={v:2d}  {40 / min(ts):7.1f} it/s (best)  "
          f"{40 / np.median(ts):7.1f} (median)")
