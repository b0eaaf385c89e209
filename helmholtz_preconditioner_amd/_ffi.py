"""ctypes loader for libhelmholtz_amd.so (the C ABI in include/helmholtz_amd.h).

There is no CPU fallback: if the HIP library is missing this module raises at
import time, and every compute call raises if the HIP runtime reports an
error (for example when no GPU is visible).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HH_LIB_PATH", os.path.join(_HERE, "libhelmholtz_amd.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"helmholtz_preconditioner_amd: native library not found at {LIB_PATH}. "
        "Build it first: python -c 'import __graft_entry__ as g; g.build()' "
        "(or `make -C helmholtz_preconditioner_amd/csrc`).")

lib = ctypes.CDLL(LIB_PATH)

# Every live handle (vectors, operators, contexts) is released by an atexit hook, vectors first:
# an object a garbage collector never finalises would otherwise still own device memory, streams
# and an RCCL communicator when the HIP runtime's own exit handlers run -- after a profiler
# (rocprofv3) has finalised its hooks, which is where such late releases crashed
# (profiles/r03i: SIGSEGV inside exit()).  Python atexit hooks run before the C runtime's.
import atexit  # noqa: E402
import weakref  # noqa: E402

_LIVE = (weakref.WeakSet(), weakref.WeakSet(), weakref.WeakSet())  # vectors, operators, contexts


def track(obj, rank: int) -> None:
    """register a handle owner for release at exit (rank 0 vector, 1 operator, 2 context)"""
    _LIVE[rank].add(obj)


def release_all() -> None:
    for live in _LIVE:
        for obj in list(live):
            try:
                obj.close()
            except Exception:  # pragma: no cover - best effort at interpreter exit
                pass


atexit.register(release_all)

c_int, c_long, c_double, c_void_p = ctypes.c_int, ctypes.c_long, ctypes.c_double, ctypes.c_void_p
c_dp = ctypes.POINTER(ctypes.c_double)
c_ip = ctypes.POINTER(ctypes.c_int)
c_lp = ctypes.POINTER(ctypes.c_long)
c_ubp = ctypes.POINTER(ctypes.c_ubyte)
PP = ctypes.POINTER(ctypes.c_void_p)

HH_PREC_NONE, HH_PREC_JACOBI, HH_PREC_SHIFTED_LAPLACE, HH_PREC_SWEEP, HH_PREC_SWEEP_REF = 0, 1, 2, 3, 4
HH_APPLY_A, HH_APPLY_JACOBI_A, HH_APPLY_PREC, HH_APPLY_PREC_A = 0, 1, 2, 3
HH_TRANSPORT_RCCL, HH_TRANSPORT_SHM = 0, 1

# callbacks return 0 to continue, non-zero to stop the solve (hh_gmres -> HH_ERR_ABORTED)
GMRES_CALLBACK = ctypes.CFUNCTYPE(c_int, c_void_p, c_long, c_double)
GMRES_CYCLE_CALLBACK = ctypes.CFUNCTYPE(c_int, c_void_p, c_long)
GMRES_HISTORY_CALLBACK = ctypes.CFUNCTYPE(c_int, c_void_p, c_long, c_int,
                                          ctypes.POINTER(ctypes.c_double))
HH_ERR_ABORTED = -6
SPAN_NAMES = ("halo", "boundary", "interior", "halo_wait", "allreduce", "column", "multidot",
              "update")  # HH_SPAN_* order (include/helmholtz_amd.h)
ABI_VERSION = 2


class HHStats(ctypes.Structure):
    _fields_ = [("solve_ms", c_double), ("inner_iterations", c_long), ("restarts", c_long),
                ("spmv_count", c_long), ("algorithmic_bytes", c_double)]


# (name, restype, argtypes) for every entry point of include/helmholtz_amd.h
SIGNATURES = [
    ("hh_abi_version", c_int, []),
    ("hh_last_error", ctypes.c_char_p, []),
    ("hh_device_count", c_int, [c_ip]),
    ("hh_comm_unique_id", c_int, [c_ubp]),
    ("hh_comm_selftest", c_int, [c_int, c_dp, c_dp]),
    ("hh_ctx_create", c_int, [c_int, c_int, c_int, c_ubp, c_int, PP]),
    ("hh_ctx_create_ex", c_int, [c_int, c_int, c_int, c_ubp, c_int, c_int, PP]),
    ("hh_ctx_destroy", c_int, [c_void_p]),
    ("hh_ctx_allreduce_max", c_int, [c_void_p, c_dp, c_int]),
    ("hh_ctx_allreduce_sum", c_int, [c_void_p, c_dp, c_int]),
    ("hh_ctx_barrier", c_int, [c_void_p]),
    ("hh_ctx_synchronize", c_int, [c_void_p]),
    ("hh_ctx_progress", c_int, [c_void_p, c_lp]),
    ("hh_knobs_json", c_int, [c_int, ctypes.c_char_p, c_int, c_ip]),
    ("hh_op_create", c_int, [c_void_p, c_int, c_int, c_double, c_double, c_double, c_double,
                             c_double, c_dp, c_double, c_double, c_double, PP]),
    ("hh_op_destroy", c_int, [c_void_p]),
    ("hh_op_local_rows", c_int, [c_void_p, c_ip, c_ip]),
    ("hh_op_set_precond", c_int, [c_void_p, c_int, c_double, c_int, c_double]),
    ("hh_op_apply", c_int, [c_void_p, c_dp, c_dp, c_int]),
    ("hh_op_diagonal", c_int, [c_void_p, c_dp]),
    ("hh_op_csr_nnz", c_int, [c_void_p, ctypes.POINTER(ctypes.c_int64)]),
    ("hh_op_export_csr", c_int, [c_void_p, c_void_p, c_void_p, c_int, c_dp, c_dp]),
    ("hh_vec_create", c_int, [c_void_p, PP]),
    ("hh_vec_destroy", c_int, [c_void_p]),
    ("hh_vec_upload", c_int, [c_void_p, c_dp]),
    ("hh_vec_download", c_int, [c_void_p, c_dp]),
    ("hh_vec_fill_hash", c_int, [c_void_p, ctypes.c_uint64]),
    ("hh_op_apply_dev", c_int, [c_void_p, c_void_p, c_void_p, c_int]),
    ("hh_op_time_apply", c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_dp, c_dp]),
    ("hh_op_time_apply_set", c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_dp,
                                     c_dp]),
    ("hh_gmres", c_int, [c_void_p, c_void_p, c_void_p, c_double, c_double, c_int, c_long, c_int,
                         c_int, c_dp, c_long, GMRES_CALLBACK, c_void_p, c_lp, c_ip, c_dp, c_dp]),
    ("hh_op_set_stencil", c_int, [c_void_p, c_int, c_double, c_double, c_double]),
    ("hh_op_set_cycle_callback", c_int, [c_void_p, GMRES_CYCLE_CALLBACK, c_void_p]),
    ("hh_op_set_history_callback", c_int, [c_void_p, GMRES_HISTORY_CALLBACK, c_void_p]),
    ("hh_op_sl_fusion", c_int, [c_void_p, c_int]),
    ("hh_op_set_krylov_mode", c_int, [c_void_p, c_int]),
    ("hh_op_set_small_cycle", c_int, [c_void_p, c_int]),
    ("hh_op_last_solve_path", c_int, [c_void_p, c_ip]),
    ("hh_op_set_timing", c_int, [c_void_p, c_int]),
    ("hh_op_read_timing", c_int, [c_void_p, c_dp, c_lp]),
    ("hh_op_small_cycle_profile", c_int, [c_void_p, c_int, c_dp]),
    ("hh_op_small_cycle_tail_profile", c_int, [c_void_p, c_dp]),
    ("hh_op_tune", c_int, [c_void_p, c_int, c_int, c_int]),
    ("hh_op_sweep_mode", c_int, [c_void_p, c_int, c_ip]),
    ("hh_op_sweep_workgroups", c_int, [c_void_p, c_int, c_ip]),
    ("hh_op_sweep_profile", c_int, [c_void_p, c_int, c_dp, c_int]),
    ("hh_tune_krylov", c_int, [c_int, c_int]),
    ("hh_op_probe_stream", c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_dp, c_ip]),
    ("hh_op_probe_stream_set", c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int,
                                       c_dp, c_ip]),
    ("hh_op_last_stats", c_int, [c_void_p, ctypes.POINTER(HHStats)]),
]

# HH_LIB_AB=1 (diagnostic A/B timing against an older build given by HH_LIB_PATH): entry points
# the older library lacks are left unbound instead of failing the import
_AB = os.environ.get("HH_LIB_AB") == "1"
for _name, _res, _args in SIGNATURES:
    if _AB and not hasattr(lib, _name):
        continue
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args

if lib.hh_abi_version() != ABI_VERSION:
    raise ImportError("libhelmholtz_amd.so ABI version mismatch")


class HHError(RuntimeError):
    """A negative hh_err code from the native library."""

    def __init__(self, code, msg):
        super().__init__(f"[hh_err {code}] {msg}")
        self.code = code


def check(rc: int) -> None:
    if rc != 0:
        raise HHError(rc, lib.hh_last_error().decode(errors="replace"))


def dptr(arr):
    """double* view of a C-contiguous float64/complex128 numpy array."""
    return arr.ctypes.data_as(c_dp)
