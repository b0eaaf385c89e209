"""Driver for PMC calibration: each streaming probe (known bytes) and the stencil, 10
launches each, at the bench workload.  Run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import helmholtz_preconditioner_amd as H  # noqa: E402
from helmholtz_preconditioner_amd import _ffi  # noqa: E402

n = 4096
om, h, eta = H.problem_params(n, 12, 100.0, 2.0)
A = H.build_A_matrix(12, 81.0, eta, om, h, n, H.marmousi_like_c_mat(n))
x, y = A.vector(), A.vector()
x.fill_hash(1)
km, bpp = ctypes.c_double(), ctypes.c_int()
for kind in (0, 1, 3, 4):
    _ffi.check(_ffi.lib.hh_op_probe_stream(A.handle, kind, 8192, x.handle, y.handle, 10,
                                           ctypes.byref(km), ctypes.byref(bpp)))
A.time_apply(x, y, 10)
print("done")
