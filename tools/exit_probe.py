"""Diagnostic for the SIGSEGV inside exit() under rocprofv3 (profiles/r03i, r04m): runs one
partitioned (cooperative-launch) or sequential sweep apply, releases every handle, writes this
process's /proc/self/maps to OUT (so the crash backtrace's addresses can be mapped to
libraries), then exits.  usage: python tools/exit_probe.py OUT [n] [workgroups] [mode]
mode: sweep (default) | smallcoop (the small-grid GMRES cycle, cooperative launch) | none"""
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import helmholtz_preconditioner_amd as H  # noqa: E402
from helmholtz_preconditioner_amd import _ffi  # noqa: E402

out = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 255
wgs = int(sys.argv[3]) if len(sys.argv) > 3 else 0
mode = sys.argv[4] if len(sys.argv) > 4 else "sweep"
om, h, eta = H.problem_params(n, 12, n / 8 + 1, 2.0)
cm, f = H.init_c1_f1(om, n)
A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm)
if mode == "sweep":
    M = H.Sweeping(A, form="thomas", workgroups=wgs)
    M.configure()
    x, y = A.vector(f.ravel()), A.vector()
    A.apply_device(x, y, _ffi.HH_APPLY_PREC)
    A.ctx.synchronize()
    print(f"sweep n={n}: partitioned={M.partitioned} workgroups={M.workgroups}", flush=True)
    x.close()
    y.close()
elif mode == "smallcoop":
    A.small_cycle("on")
    H.gmres(A, f.ravel(), rtol=1e-3, restart=20, maxiter=20)
    print("small cycle:", A.last_solve_path(), flush=True)
A.close()
H.default_context().close()
shutil.copyfile("/proc/self/maps", out)
print("maps written; exiting", flush=True)
