"""Sweeping preconditioner (row F1) timings on the device vs the reference's SuperLU path
(oracle restatement of algo2_3 / algo2_4 on this host's CPU).
usage: python tools/bench_sweep.py [n ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import helmholtz_preconditioner_amd as H  # noqa: E402
from helmholtz_preconditioner_amd import _ffi  # noqa: E402

ns = [int(v) for v in sys.argv[1:]] or [127, 255, 511, 1023]
for n in ns:
    b, C, wn = 12, {127: 81.0, 255: 62.0, 511: 81.0, 1023: 100.0}.get(n, 81.0), n // 8 + 1
    om, h, eta = H.problem_params(n, b, float(wn), 2.0)
    cm, f = H.init_c1_f1(om, n)
    A = H.build_A_matrix(b, C, eta, om, h, n, cm)
    A.ctx.synchronize()
    t0 = time.perf_counter()
    A.set_preconditioner(_ffi.HH_PREC_SWEEP)
    t_setup = time.perf_counter() - t0
    x, y = A.vector(f.ravel()), A.vector()
    A.apply_device(x, y, _ffi.HH_APPLY_PREC)
    t0 = time.perf_counter()
    for _ in range(2):
        A.apply_device(x, y, _ffi.HH_APPLY_PREC)
    t_apply = (time.perf_counter() - t0) / 2
    t0 = time.perf_counter()
    u, info, hist = H.gmres(A, f.ravel(), rtol=1e-3, restart=20, maxiter=300, M=H.Sweeping(A),
                            callback=lambda r: None, callback_type="legacy", return_history=True)
    t_solve = time.perf_counter() - t0
    line = (f"n={n} b={b} wn={wn}: setup {t_setup*1e3:.1f} ms, apply {t_apply*1e3:.1f} ms, "
            f"corrected-sweep GMRES {len(hist)} its info={info} in {t_solve:.3f} s")
    if n <= 255 and os.path.isdir(os.path.join(ROOT, "oracle")):
        from oracle import helmholtz_oracle as O
        t0 = time.perf_counter()
        st = O.SweepState(b, C, eta, om, h, n, cm)
        cpu_setup = time.perf_counter() - t0
        t0 = time.perf_counter()
        st.apply(f.ravel(), corrected=True)
        cpu_apply = time.perf_counter() - t0
        line += f" | CPU SuperLU (1 core): setup {cpu_setup:.2f} s, apply {cpu_apply*1e3:.0f} ms"
    print(line, flush=True)
    del A, x, y
