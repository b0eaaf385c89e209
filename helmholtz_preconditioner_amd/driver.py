"""The reference's experiment harness on the device path.

Reference: ``gmres_counter`` (code.py:411-420) and ``run_solver(n, b, wave_num, const,
alpha, init_func=init_c1_f1, plot_solution=True) -> (init_time, solve_time)``
(code.py:424-541): omega = 2 pi wave_num + i alpha, h = 1/(n+1), eta = b h; build A;
set up the sweeping moving-PML preconditioner (algo2_3); GMRES(rtol=1e-3) with it; time
"init" (assembly + preconditioner setup) and "solve" separately; optionally plot
flipud(Re u).

Here every step runs on the GPU.  ``preconditioner`` selects the M slot:

* ``"sweep-asis"`` (default) -- exactly what run_solver runs: M x = algo2_4(f) for every x
  and the middle sweep u -= T u (quirks Q1/Q2).  Same iteration counts and
  (non-)solutions as the reference.
* ``"sweep"`` -- Engquist-Ying Alg. 2.4 with both quirks corrected (converges).
* ``"shifted-laplace"``, ``"jacobi"``, ``None`` -- the build-side preconditioners of
  BASELINE configs 1-3.
"""
from __future__ import annotations

import time

import numpy as np

from .media import init_c1_f1, problem_params
from .operator import ShiftedLaplace, Sweeping, build_A_matrix
from .solver import gmres


class gmres_counter:
    """Counts GMRES callbacks (= inner iterations with the legacy callback), code.py:411-420."""

    def __init__(self, disp=True):
        self._disp = disp
        self.niter = 0

    def __call__(self, rk=None):
        self.niter += 1
        if self._disp:
            print('iter %3i\trk = %s' % (self.niter, str(rk)))


def _make_M(A, preconditioner):
    if preconditioner is None or preconditioner == "none":
        return None
    if preconditioner == "sweep-asis":
        return Sweeping(A, reference=True)
    if preconditioner == "sweep":
        return Sweeping(A, reference=False)
    if preconditioner == "shifted-laplace":
        return ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7)
    if preconditioner == "jacobi":
        return "jacobi"
    raise ValueError(f"unknown preconditioner {preconditioner!r}")


def run_solver(n, b, wave_num, const, alpha, init_func=init_c1_f1, plot_solution=True, *,
               preconditioner="sweep-asis", rtol=1e-3, restart=20, maxiter=None, verbose=True,
               plot_path=None, context=None, return_details=False):
    """Drop-in for ``run_solver`` (code.py:424): returns ``(init_time, solve_time)``
    (plus a details dict with ``return_details=True``: u, info, iterations)."""
    counter_prec = gmres_counter(False)
    t0 = time.time()
    omega, h, eta = problem_params(n, b, wave_num, alpha)        # code.py:442-444
    c_mat, f_mat = init_func(omega, n)                           # code.py:447
    f_vec = f_mat.flatten()                                      # code.py:448
    A = build_A_matrix(b, const, eta, omega, h, n, c_mat, context=context)
    M = _make_M(A, preconditioner)
    if hasattr(M, "configure"):
        M.configure()  # algo2_3: every factorisation happens in "init", as in the reference
        A.ctx.synchronize()
    t1 = time.time()
    u, exit_code = gmres(A, f_vec, M=M, rtol=rtol, restart=restart, maxiter=maxiter,
                         callback=counter_prec, callback_type="legacy")
    t2 = time.time()
    if verbose:
        print("GMRES iterations with preconditioner: " + str(counter_prec.niter))
        print("Initialization time = " + str(t1 - t0))
        print("GMRES solve time = " + str(t2 - t1))
    if plot_solution or plot_path is not None:
        from .io import plot_solution as _plot
        _plot(u, n, wave_num, const, path=plot_path)
    if return_details:
        return t1 - t0, t2 - t1, dict(u=u, info=exit_code, iterations=counter_prec.niter,
                                      omega=omega, h=h, eta=eta)
    return t1 - t0, t2 - t1


def true_relative_residual(A, u, f):
    """||f - A u|| / ||f|| on the device operator (host vectors)."""
    r = np.asarray(f) - A @ np.asarray(u)
    return float(np.linalg.norm(r) / np.linalg.norm(f))
