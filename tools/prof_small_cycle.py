"""Where the time of the small-grid whole-cycle GMRES kernel goes (BASELINE config 1 by default):
per-phase wall-clock totals of workgroup 0 (hh_op_small_cycle_profile) per inner iteration, and
the solve's iterations per second with the kernel on and off.
usage: python tools/prof_small_cycle.py [--n 128] [--iters 200] [--precond none|jacobi]"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import helmholtz_preconditioner_amd as H  # noqa: E402
from helmholtz_preconditioner_amd import _ffi  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=128)
p.add_argument("--iters", type=int, default=200)
p.add_argument("--wave-num", type=float, default=8.0)
p.add_argument("--precond", default="none")
p.add_argument("--cb", default="lambda", choices=["lambda", "none"],
               help="legacy callback (as bench.py) or none (host cost of the callback)")
a = p.parse_args()
n = a.n
om, h, eta = H.problem_params(n, 12, a.wave_num, 2.0)
A = H.build_A_matrix(12, 81.0, eta, om, h, n, H.constant_c_mat(n))
f = A.vector(H.init_f1_mat(.5, .125, om, n).ravel())
M = None if a.precond == "none" else "jacobi"
for mode in ("on", "off", "on"):
    A.small_cycle(mode)
    H.gmres(A, f, rtol=1e-14, restart=20, maxiter=20, M=M, callback=lambda r: None,
            callback_type="legacy")
    ph = (ctypes.c_double * 8)()
    _ffi.check(_ffi.lib.hh_op_small_cycle_profile(A.handle, 1, ph))
    t0 = time.perf_counter()
    if a.cb == "lambda":
        H.gmres(A, f, rtol=1e-14, restart=20, maxiter=a.iters, M=M, callback=lambda r: None,
                callback_type="legacy")
    else:  # (maxiter then counts cycles: iters // 20 of them)
        H.gmres(A, f, rtol=1e-14, restart=20, maxiter=a.iters // 20, M=M)
    dt = time.perf_counter() - t0
    tail = (ctypes.c_double * 8)()
    if mode == "on":
        _ffi.check(_ffi.lib.hh_op_small_cycle_tail_profile(A.handle, tail))
    _ffi.check(_ffi.lib.hh_op_small_cycle_profile(A.handle, 0, ph))
    per = [ph[q] / a.iters for q in (0, 5, 6, 1, 3, 2, 4)]
    span = sum(ph[q] for q in range(7))
    mhz = ph[7] / span if span > 0 else 0.0
    print(f"n={n} small_cycle={mode}: {a.iters / dt:9.1f} it/s ({dt / a.iters * 1e6:6.2f} us/it)"
          + ("" if mode == "off" else
             "  phases us/it: stencil %.2f dots %.2f publish %.2f allreduce %.2f coef+ghosts %.2f"
             " update %.2f givens-wait %.2f  (shader clock %.0f MHz)"
             % tuple(per + [mhz])), flush=True)
    if mode == "on":
        cyc = -(-a.iters // 20)
        print("  per cycle (us, workgroup 0): head %.2f  last round + Givens solve %.2f  x update +"
              " hand-off %.2f  residual + all-reduce %.2f\n  Givens workgroup per cycle: waits %.2f"
              "  per-round work %.2f  last column + solve + publish %.2f" % tuple(v / cyc for v in tail[:7]),
              flush=True)
        print("  all-reduce first hop (publish -> column 0 reduced on workgroup 0): %.2f us/it"
              % (tail[7] / a.iters),
              flush=True)

for rep in range(2):  # the profiled runs instrument workgroup 0; then the same without it
    A.small_cycle("on")
    H.gmres(A, f, rtol=1e-14, restart=20, maxiter=20, M=M, callback=lambda r: None,
            callback_type="legacy")
    t0 = time.perf_counter()
    H.gmres(A, f, rtol=1e-14, restart=20, maxiter=a.iters, M=M, callback=lambda r: None,
            callback_type="legacy")
    dt = time.perf_counter() - t0
    print(f"n={n} small_cycle=on, not profiled: {a.iters / dt:9.1f} it/s"
          f" ({dt / a.iters * 1e6:6.2f} us/it)", flush=True)
