"""Sweeping preconditioner (row F1) timings on the device vs the reference's SuperLU path
(oracle restatement of algo2_3 / algo2_4 on this host's CPU).
usage: python tools/bench_sweep.py [--form dense|thomas|thomas-sequential|auto] [--maxiter K]
                                   [--wgs G] [n ...]
--maxiter 0 skips the GMRES solve (default 300; large n with the solve forms takes ~1 s/apply)

Dense-form apply algorithmic bytes: every transfer matrix read once by the fused
forward+middle pass and once by the backward pass: 2 (n - b) n^2 16 B + b n^2 16 B (F0)
+ n^2 16 B (FC), i.e. the GEMV chain's matrix stream (vectors ignored)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import helmholtz_preconditioner_amd as H  # noqa: E402
from helmholtz_preconditioner_amd import _ffi  # noqa: E402

def device_used_bytes():
    """bytes in use on the current device (hipMemGetInfo: total - free), for the peak-memory
    figure of the preconditioner's operator data"""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    free, total = ctypes.c_size_t(), ctypes.c_size_t()
    if hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) != 0:
        return None
    return total.value - free.value


args = sys.argv[1:]
form, maxiter, wgs = "auto", 300, 0
while args and args[0].startswith("--"):
    if args[0] == "--form":
        form = args[1]
    elif args[0] == "--maxiter":
        maxiter = int(args[1])
    elif args[0] == "--wgs":
        wgs = int(args[1])
    args = args[2:]
ns = [int(v) for v in args] or [127, 255, 511, 1023]
for n in ns:
    b, C, wn = 12, {127: 81.0, 255: 62.0, 511: 81.0, 1023: 100.0}.get(n, 81.0), n // 8 + 1
    om, h, eta = H.problem_params(n, b, float(wn), 2.0)
    cm, f = H.init_c1_f1(om, n)
    A = H.build_A_matrix(b, C, eta, om, h, n, cm)
    A.ctx.synchronize()
    mem0 = device_used_bytes()
    t0 = time.perf_counter()
    Msw = H.Sweeping(A, form=form, workgroups=wgs)
    Msw.configure()
    A.ctx.synchronize()
    t_setup = time.perf_counter() - t0
    mem1 = device_used_bytes()
    x, y = A.vector(f.ravel()), A.vector()
    A.apply_device(x, y, _ffi.HH_APPLY_PREC)
    A.ctx.synchronize()
    mem2 = device_used_bytes()  # (+ the apply's workspaces and the two vectors)
    t0 = time.perf_counter()
    reps = 10 if Msw.dense or n <= 1023 else 2
    for _ in range(reps):
        A.apply_device(x, y, _ffi.HH_APPLY_PREC)
    A.ctx.synchronize()
    t_apply = (time.perf_counter() - t0) / reps
    hist, info, t_solve = [], None, 0.0
    if maxiter > 0:
        t0 = time.perf_counter()
        u, info, hist = H.gmres(A, f.ravel(), rtol=1e-3, restart=20, maxiter=maxiter, M=Msw,
                                callback=lambda r: None, callback_type="legacy",
                                return_history=True)
        t_solve = time.perf_counter() - t0
    gbs = ""
    if Msw.dense:
        alg = (2 * (n - b) + b + 1) * n * n * 16
        gbs = f" ({alg / t_apply / 1e9:.0f} GB/s algorithmic, dense)"
    kind = "dense" if Msw.dense else (f"partitioned, {Msw.workgroups} workgroups" if Msw.partitioned
                                      else "sequential")
    x.close()  # (every handle released explicitly, before the next grid and before exit)
    y.close()
    A.close()
    line = (f"n={n} b={b} wn={wn} form={form} ({kind}): setup {t_setup*1e3:.1f} ms, apply {t_apply*1e3:.2f} ms{gbs}, "
            f"corrected-sweep GMRES {len(hist)} its info={info} in {t_solve:.3f} s")
    if mem0 is not None and mem1 is not None:
        line += (f" | device memory: operator {mem0 / 1e9:.2f} GB, + preconditioner "
                 f"{(mem1 - mem0) / 1e9:.2f} GB = {mem1 / 1e9:.2f} GB in use after setup, "
                 f"{mem2 / 1e9:.2f} GB after the first apply")
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
H.default_context().close()  # (the last handle, before exit)
