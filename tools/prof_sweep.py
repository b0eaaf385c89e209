"""Phase timing of the partitioned block-Thomas sweeps (hh_op_sweep_profile): per solve, in
microseconds of each workgroup's thread-0 wall clock, for workgroup 0 and the max over
workgroups.  usage: python tools/prof_sweep.py [--wgs G] [--reps R] [n ...]"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import helmholtz_preconditioner_amd as H  # noqa: E402
from helmholtz_preconditioner_amd import _ffi  # noqa: E402

args = sys.argv[1:]
wgs, reps = 0, 4
while args and args[0].startswith("--"):
    if args[0] == "--wgs":
        wgs = int(args[1])
    elif args[0] == "--reps":
        reps = int(args[1])
    args = args[2:]
NAMES = ["local fwd", "stage f", "chain0+pub|poll f", "grid+chain f", "fixup+local bwd",
         "stage b", "chain0+pub|poll b", "grid+chain b", "fixup+out"]
for n in [int(v) for v in args] or [1023]:
    b = 12
    om, h, eta = H.problem_params(n, b, float(n // 8 + 1), 2.0)
    cm, f = H.init_c1_f1(om, n)
    A = H.build_A_matrix(b, 81.0, eta, om, h, n, cm)
    M = H.Sweeping(A, form="thomas", workgroups=wgs)
    M.configure()
    x, y = A.vector(f.ravel()), A.vector()
    A.apply_device(x, y, _ffi.HH_APPLY_PREC)
    A.ctx.synchronize()
    _ffi.check(_ffi.lib.hh_op_sweep_profile(A.handle, 1, None, 0))
    t0 = time.perf_counter()
    for _ in range(reps):
        A.apply_device(x, y, _ffi.HH_APPLY_PREC)
    A.ctx.synchronize()
    t_apply = (time.perf_counter() - t0) / reps
    out = (ctypes.c_double * (64 * 16))()
    _ffi.check(_ffi.lib.hh_op_sweep_profile(A.handle, 0, out, 64 * 16))
    G = M.workgroups
    ph = np.array(out[:G * 16]).reshape(G, 16)[:, :9]
    solves = reps * 2 * (n - b + 1)  # forward + backward sweeps, one H_F solve each
    per = ph / solves
    print(f"n={n} G={G}: apply {t_apply * 1e3:.2f} ms, {solves // reps} partitioned solves per "
          f"apply = {t_apply / (solves / reps) * 1e6:.1f} us per solve; phases per solve (us):",
          flush=True)
    for k, nm in enumerate(NAMES):
        print(f"  {nm:20s} wg0 {per[0, k]:6.2f}  max {per[:, k].max():6.2f}  min {per[:, k].min():6.2f}")
    print(f"  {'sum':20s} wg0 {per[0].sum():6.2f}", flush=True)
    del A, M, x, y
