"""MI355X-native Helmholtz operator apply and GMRES solve.

Drop-in for the hot path of bocchs/helmholtz-preconditioner (code.py):

    from helmholtz_preconditioner_amd import build_A_matrix, gmres, init_c1_f1
    omega, h, eta = problem_params(n, b, wave_num, alpha)          # code.py:442-444
    c_mat, f_mat = init_c1_f1(omega, n)                             # code.py:447
    A = build_A_matrix(b, const, eta, omega, h, n, c_mat)           # code.py:450
    u, exit_code = gmres(A, f_mat.flatten(), M='jacobi', rtol=1e-3) # code.py:516

The kernels are hand-written HIP for gfx950 in ``csrc/`` and are reached through
the C ABI in ``include/helmholtz_amd.h`` (ctypes shim ``_ffi.py``).  Importing
this package fails if that library has not been built; there is no CPU path.
"""
from ._ffi import HHError  # noqa: F401  (raises ImportError if the .so is missing)
from .context import Context, default_context, device_count, knobs, set_default_context, unique_id  # noqa: F401,E501
from .media import (constant_c_mat, init_c1_f1, init_c1_f2, init_c1_mat, init_c2_f1,  # noqa: F401
                    init_c2_f2, init_c2_mat, init_f1_mat, init_f1_rows, init_f2_mat, marmousi_like_c_mat,
                    problem_params)
from .operator import (DeviceOperator, DevicePreconditioner, DeviceVector, Jacobi,  # noqa: F401
                       ShiftedLaplace, STENCIL9_WEIGHTS, Sweeping, build_A_matrix)
from .solver import gmres  # noqa: F401
from .driver import gmres_counter, run_solver, true_relative_residual  # noqa: F401
from .io import (load_c_mat, load_solution, load_velocity_model, plot_solution,  # noqa: F401
                 resample_velocity, save_c_mat, save_solution, solution_image)
from . import dist  # noqa: F401

__all__ = [
    "build_A_matrix", "gmres", "DeviceOperator", "DeviceVector", "Jacobi", "ShiftedLaplace",
    "Sweeping", "STENCIL9_WEIGHTS",
    "Context", "default_context", "set_default_context", "device_count", "unique_id", "knobs",
    "init_c1_mat", "init_c2_mat", "init_f1_mat", "init_f1_rows", "init_f2_mat", "init_c1_f1", "init_c1_f2",
    "init_c2_f1", "init_c2_f2", "constant_c_mat", "marmousi_like_c_mat", "problem_params",
    "HHError", "run_solver", "gmres_counter", "true_relative_residual",
    "load_c_mat", "save_c_mat", "load_velocity_model", "resample_velocity", "save_solution",
    "load_solution", "solution_image", "plot_solution",
]
