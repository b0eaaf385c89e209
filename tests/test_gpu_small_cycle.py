"""GPU tier: the whole-cycle GMRES kernel for small grids (csrc/gmres_small.hip; BASELINE
config 1 runs on it) against the reference's own histories (tests/golden: scipy gmres as
code.py:516 calls it) to the 1e-6 contract, and against the regular five-launch cycle.

Covered: config 1 itself (128^2, no preconditioner, K = 200 inner iterations: ten restart
cycles), Jacobi, a converging run (adaptive ptol, several cycles, info 0), nonzero x0, legacy
maxiter ending inside a cycle, restart 1 and 7, ragged n (block sizes not a multiple of the
wave, one-row grids), both media kinds.
"""
import os
import tempfile

import numpy as np
import pytest

import helmholtz_preconditioner_amd as H
from conftest import load_golden, medium, rand_complex
from oracle import helmholtz_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope="module")
def ctx():
    return H.Context(device=0)


def relerr(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


@pytest.mark.parametrize("name", ["gmres_n128_none.npz", "gmres_n128_jacobi.npz",
                                  "gmres_n64_c1_none.npz"])
def test_small_cycle_matches_reference_golden(ctx, name):
    z = load_golden(name)
    n = int(z["n"])
    om = complex(z["omega"])
    A = H.build_A_matrix(int(z["b"]), float(z["C"]), float(z["eta"]), om, float(z["h"]), n,
                         medium(str(z["medium"]), n), context=ctx)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    M = "jacobi" if str(z["precond"]) == "jacobi" else None
    out = {}
    for mode in ("on", "off"):
        A.small_cycle(mode)
        hist = []
        x, info = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=int(z["K"]), M=M,
                          callback=hist.append, callback_type='legacy')
        out[mode] = (x, info, np.array(hist))
    A.small_cycle("auto")
    x, info, hist = out["on"]
    assert info == int(z["info"]) and len(hist) == int(z["niter"])
    assert np.max(np.abs(hist - z["history"]) / z["history"]) < TOL
    assert relerr(x, z["x"]) < TOL
    xo, _, ho = out["off"]  # (other summation order, lagged normalisation: rounding only)
    assert np.max(np.abs(hist - ho) / ho) < 1e-9
    assert relerr(x, xo) < 1e-9


@pytest.mark.parametrize("n,kind,precond,restart,K", [
    (37, "c1", None, 20, 45), (63, "c2", "jacobi", 7, 30), (65, "const", None, 1, 6),
    (1, "const", None, 20, 3), (2, "c1", "jacobi", 20, 3), (200, "c1", "jacobi", 20, 25),
    (128, "const", None, 23, 50)])
def test_small_cycle_matches_regular_cycle(ctx, n, kind, precond, restart, K):
    b, C, wn = min(6, max(1, n // 4)), 61.0, 3.0
    om, h, eta = O.problem_params(n, b, wn, 2.0)
    cm = medium(kind, n)
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    out = []
    for mode in ("on", "off"):
        A.small_cycle(mode)
        x, info, hist = H.gmres(A, f, rtol=1e-3, restart=restart, maxiter=K, M=precond,
                                callback=lambda r: None, callback_type="legacy",
                                return_history=True)
        out.append((x, info, hist))
    (x1, i1, h1), (x2, i2, h2) = out
    assert i1 == i2 and len(h1) == len(h2)
    assert np.all(np.abs(h1 - h2) <= 1e-9 * np.abs(h2) + 1e-15)  # (n = 1: presid 0)
    assert np.linalg.norm(x1 - x2) <= 1e-9 * np.linalg.norm(x2)


def test_small_cycle_converging_and_x0(ctx):
    n, b, C, wn, al = 40, 6, 61.0, 1.0, 2.0
    cm = medium("c2", n)
    om, h, eta = O.problem_params(n, b, wn, al)
    Aref = O.build_A_matrix(b, C, eta, om, h, n, cm)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    A.small_cycle("on")
    xr, infor, histr, _ = O.gmres_reference(Aref, f, M=O.jacobi_preconditioner(Aref), rtol=1e-4,
                                            restart=10, maxiter=400)
    x, info, hist = H.gmres(A, f, rtol=1e-4, restart=10, maxiter=400, M="jacobi",
                            callback=lambda r: None, callback_type='legacy', return_history=True)
    assert info == infor == 0 and len(hist) == len(histr)
    assert np.max(np.abs(hist - histr) / histr) < TOL
    assert relerr(x, xr) < TOL
    x0 = 1e-3 * rand_complex(n * n, 9)
    xr0, infor0, histr0, _ = O.gmres_reference(Aref, f, rtol=1e-3, restart=20, maxiter=60,
                                               x0=x0.copy())
    x5, info5, hist5 = H.gmres(A, f, x0=x0, rtol=1e-3, restart=20, maxiter=60,
                               callback=lambda r: None, callback_type='legacy',
                               return_history=True)
    assert info5 == infor0 and len(hist5) == len(histr0)
    assert np.max(np.abs(hist5 - histr0) / histr0) < TOL
    assert relerr(x5, xr0) < TOL


@pytest.mark.parametrize("case", ["cycles", "converge", "xcb"])
def test_small_cycle_queued_cycles(ctx, case):
    """Whole-cycle launches are queued several at a time, scipy's restart-loop decisions taken
    on the device (runtime.cpp kSmallBatch): maxiter counting restart cycles across batches, a
    solve that converges inside a batch (the launches queued behind it return at once, and the
    next solve starts clean), and the x callback (one cycle per batch) -- all as the regular
    cycle runs them."""
    n, b, C, wn = 48, 6, 61.0, 2.0
    om, h, eta = O.problem_params(n, b, wn, 2.0)
    A = H.build_A_matrix(b, C, eta, om, h, n, medium("c2", n), context=ctx)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    kw = {"cycles": dict(rtol=1e-12, restart=5, maxiter=19),  # (16 + 3: two batches)
          "converge": dict(rtol=1e-4, restart=10, maxiter=400, M="jacobi"),
          "xcb": dict(rtol=1e-4, restart=10, maxiter=400, M="jacobi")}[case]
    out = []
    for mode in ("on", "off"):
        A.small_cycle(mode)
        calls = []
        if case == "xcb":
            x, info = H.gmres(A, f, callback=lambda xk: calls.append(np.array(xk)),
                              callback_type="x", **kw)
            hist = None
        else:
            x, info, hist = H.gmres(A, f, callback=lambda r: None, callback_type="pr_norm",
                                    return_history=True, **kw)
        out.append((x, info, hist, calls))
        if case == "converge":  # a second solve after the skipped launches: same again
            x2, info2, hist2 = H.gmres(A, f, callback=lambda r: None, callback_type="pr_norm",
                                       return_history=True, **kw)
            assert info2 == info and np.array_equal(hist2, hist) and np.array_equal(x2, x)
    A.small_cycle("auto")
    (x1, i1, h1, c1), (x2, i2, h2, c2) = out
    assert i1 == i2
    if case == "cycles":
        assert i1 == 19 and len(h1) == len(h2) == 95, (i1, len(h1), len(h2))
    if case == "converge":
        assert i1 == 0 and len(h1) == len(h2) and len(h1) > 10
    if h1 is not None:
        # (hundreds of iterations in two summation orders: rounding grows past 1e-9 -- the
        # 1e-6 contract of DESIGN 6)
        assert np.all(np.abs(h1 - h2) <= 1e-6 * np.abs(h2))
    if case == "xcb":
        assert len(c1) == len(c2) > 4
        for u, v in zip(c1, c2):
            assert np.linalg.norm(u - v) <= 1e-6 * np.linalg.norm(v)
    assert np.linalg.norm(x1 - x2) <= 1e-6 * np.linalg.norm(x2)


@pytest.mark.parametrize("wide", ["1", "4"])
def test_small_cycle_block_widths(wide):
    """The whole-cycle kernel with 1 and 4 copies of the row's threads (HH_SMALL_WIDE; 4 takes
    the row-split basis update) against the regular cycle, in a child process (the width is read
    once per process)."""
    import subprocess
    import sys
    code = r'''
import numpy as np, sys
sys.path.insert(0, ".")
import helmholtz_preconditioner_amd as H
from oracle import helmholtz_oracle as O
for n, pre in ((128, None), (37, "jacobi"), (65, None)):
    om, h, eta = O.problem_params(n, 6, 3.0, 2.0)
    A = H.build_A_matrix(6, 61.0, eta, om, h, n, H.init_c1_mat(.5, .5, n))
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    out = []
    for mode in ("on", "off"):
        A.small_cycle(mode)
        out.append(H.gmres(A, f, rtol=1e-3, restart=20, maxiter=45, M=pre,
                           callback=lambda r: None, callback_type="legacy", return_history=True))
    (x1, i1, h1), (x2, i2, h2) = out
    assert i1 == i2 and len(h1) == len(h2), (n, i1, i2)
    # (three restart cycles in two summation orders: the 1e-6 contract of DESIGN 6)
    assert np.all(np.abs(h1 - h2) <= 1e-6 * np.abs(h2) + 1e-15), n
    assert np.linalg.norm(x1 - x2) <= 1e-6 * np.linalg.norm(x2), n
print("ok")
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HH_SMALL_WIDE=wide)
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_small_cycle_path_reported(ctx):
    """The operator reports which cycle form ran (hh_op_last_solve_path)."""
    n = 64
    om, h, eta = O.problem_params(n, 6, 3.0, 2.0)
    A = H.build_A_matrix(6, 61.0, eta, om, h, n, medium("c1", n), context=ctx)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    for mode, path in (("on", "small-cycle"), ("off", "regular"), ("auto", "small-cycle")):
        A.small_cycle(mode)
        H.gmres(A, f, rtol=1e-3, restart=20, maxiter=25, callback=lambda r: None,
                callback_type="legacy")
        assert A.last_solve_path() == path, (mode, A.last_solve_path())
    n = 240  # ineligible: 3 n (restart + 1) x 16 B of basis exceed the LDS -> regular cycle
    om, h, eta = O.problem_params(n, 6, 3.0, 2.0)
    A = H.build_A_matrix(6, 61.0, eta, om, h, n, medium("c1", n), context=ctx)
    A.small_cycle("on")
    H.gmres(A, O.init_f1_mat(.5, .125, om, n).ravel(), rtol=1e-3, restart=20, maxiter=25,
            callback=lambda r: None, callback_type="legacy")
    assert A.last_solve_path() == "regular"


def test_small_cycle_refused_launch_falls_back():
    """A grid the kernel's co-residency gate refuses (simulated: HH_SMALL_COOP_REFUSE=1 makes
    workgroup 0 decide ABORT, as when its co-residents never arrive) leaves before touching any
    state, and the whole solve runs on the regular cycle -- no spin to a timeout, no partial
    state -- with the reference's history (golden, 1e-6).  Child process: the knob is read once
    per process."""
    import subprocess
    import sys
    code = r'''
import numpy as np, sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import helmholtz_preconditioner_amd as H
from conftest import load_golden, medium
from oracle import helmholtz_oracle as O
z = load_golden("gmres_n128_none.npz")
n = int(z["n"]); om = complex(z["omega"])
A = H.build_A_matrix(int(z["b"]), float(z["C"]), float(z["eta"]), om, float(z["h"]), n,
                     medium(str(z["medium"]), n))
f = O.init_f1_mat(.5, .125, om, n).ravel()
A.small_cycle("on")
x, info, hist = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=int(z["K"]),
                        callback=lambda r: None, callback_type="legacy", return_history=True)
assert A.last_solve_path() == "small-cycle refused -> regular", A.last_solve_path()
assert info == int(z["info"]) and len(hist) == int(z["niter"])
assert np.max(np.abs(hist - z["history"]) / z["history"]) < 1e-6
assert np.linalg.norm(x - z["x"]) < 1e-6 * np.linalg.norm(z["x"])
print("ok")
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HH_SMALL_COOP_REFUSE="1")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("precond", [None, "jacobi"])
@pytest.mark.parametrize("cbtype", ["legacy", "pr_norm"])
def test_small_cycle_refusal_after_cycles_hands_over(precond, cbtype):
    """A refusal after cycles have run (simulated: HH_SMALL_REFUSE_AT=2 makes the gate refuse the
    solve's second launch, after the first batch of 16 restart cycles) hands the solve to the
    regular cycle at that restart boundary -- x, V[0] = M r, |r|^2, |M r|^2 (Jacobi: its own
    report slot) and the device's ptol state as the last completed cycle left them -- instead
    of failing: same info and history (1e-9) as the uninterrupted small-cycle solve, for M none
    and Jacobi, in legacy mode (maxiter caps inner iterations) and in the restart-loop mode of
    pr_norm (maxiter caps cycles; ptol and its growth factor read back from the device).  Child
    processes: the knob is read once per process."""
    import subprocess
    import sys
    code = r'''
import numpy as np, sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import helmholtz_preconditioner_amd as H
from conftest import medium
from oracle import helmholtz_oracle as O
n, b, C, wn = 37, 6, 61.0, 3.0
om, h, eta = O.problem_params(n, b, wn, 2.0)
A = H.build_A_matrix(b, C, eta, om, h, n, medium("c1", n))
f = O.init_f1_mat(.5, .125, om, n).ravel()
A.small_cycle("on")
M = None if sys.argv[2] == "none" else sys.argv[2]
cb = sys.argv[3]
x, info, hist = H.gmres(A, f, rtol=1e-10, restart=2, maxiter=40 if cb == "legacy" else 20, M=M,
                        callback=lambda r: None, callback_type=cb, return_history=True)
np.savez(sys.argv[1], x=x, info=info, hist=hist, path=A.last_solve_path())
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = []
    with tempfile.TemporaryDirectory() as td:
        for at in ("0", "2"):
            out = os.path.join(td, f"r{at}.npz")
            env = dict(os.environ, HH_SMALL_REFUSE_AT=at)
            r = subprocess.run([sys.executable, "-c", code, out, precond or "none", cbtype],
                               cwd=root, env=env, capture_output=True, text=True, timeout=240)
            assert r.returncode == 0, r.stdout + r.stderr
            res.append(np.load(out))
    a, b = res
    assert str(a["path"]) == "small-cycle" and str(b["path"]) == "small-cycle refused -> regular"
    assert int(a["info"]) == int(b["info"]) and len(a["hist"]) == len(b["hist"]) >= 40
    assert np.array_equal(a["hist"][:32], b["hist"][:32])  # (the 16 cycles before the refusal)
    assert np.all(np.abs(a["hist"] - b["hist"]) <= 1e-9 * np.abs(a["hist"]) + 1e-15)
    assert np.linalg.norm(a["x"] - b["x"]) <= 1e-9 * np.linalg.norm(a["x"])
