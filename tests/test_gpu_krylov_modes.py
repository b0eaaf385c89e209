"""GPU tier: the one-allreduce GMRES iteration (hh_op_set_krylov_mode 2, lagged normalisation;
the default across ranks) forced on a single rank, against the reference's own histories
(tests/golden, scipy gmres as code.py:516 calls it) and the oracle -- the same 1e-6 contract as
the two-allreduce path -- and against the two-allreduce path itself.

Covered: stagnating runs at restart boundaries (legacy maxiter inside a cycle), a converging
run with adaptive ptol and several restart cycles, a nonzero x0, all three preconditioners,
breakdown (zero right-hand side in a cycle), callback types.
"""
import os

import numpy as np
import pytest

import helmholtz_preconditioner_amd as H
from conftest import ROOT, load_golden, medium, rand_complex
from oracle import helmholtz_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope="module")
def ctx():
    c = H.Context(device=0)
    yield c


def relerr(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


@pytest.mark.parametrize("name", ["gmres_n128_none.npz", "gmres_n128_jacobi.npz",
                                  "gmres_n64_c1_none.npz"])
def test_one_allreduce_matches_reference_golden(ctx, name):
    z = load_golden(name)
    n = int(z["n"])
    om = complex(z["omega"])
    cm = medium(str(z["medium"]), n)
    A = H.build_A_matrix(int(z["b"]), float(z["C"]), float(z["eta"]), om, float(z["h"]), n, cm,
                         context=ctx)
    A.krylov_mode("one")
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    M = "jacobi" if str(z["precond"]) == "jacobi" else None
    hist = []
    x, info = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=int(z["K"]), M=M,
                      callback=hist.append, callback_type='legacy')
    hist = np.array(hist)
    assert info == int(z["info"]) and len(hist) == int(z["niter"])
    assert np.max(np.abs(hist - z["history"]) / z["history"]) < TOL
    assert relerr(x, z["x"]) < TOL


@pytest.mark.parametrize("precond", ["none", "jacobi", "sl"])
@pytest.mark.parametrize("restart,K", [(20, 45), (7, 30), (1, 6)])
def test_one_allreduce_matches_two_allreduce(ctx, precond, restart, K):
    """same histories and fields as the exact-normalisation path to rounding (1e-10), with
    legacy maxiter ending inside a cycle and at a cycle edge; restart 1 (a single column per
    cycle: only the final lagged step)"""
    n, b, C, wn = 96, 12, 81.0, 6.0
    om, h, eta = O.problem_params(n, b, wn, 2.0)
    cm = medium("c1", n)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    M = {"none": None, "jacobi": "jacobi",
         "sl": H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7)}[precond]
    out = []
    for mode in ("two", "one"):
        A.krylov_mode(mode)
        x, info, hist = H.gmres(A, f, rtol=1e-3, restart=restart, maxiter=K, M=M,
                                callback=lambda r: None, callback_type="legacy",
                                return_history=True)
        out.append((x, info, hist))
    A.krylov_mode("auto")
    (x2, i2, h2), (x1, i1, h1) = out
    assert i1 == i2 and len(h1) == len(h2) == K
    assert np.max(np.abs(h1 - h2) / h2) < 1e-10
    assert relerr(x1, x2) < 1e-10


def test_one_allreduce_converging_cycles_and_x0(ctx):
    """a converging run (info 0, several restart cycles, adaptive ptol, pr_norm counting) and a
    nonzero x0, against scipy"""
    import scipy.sparse.linalg
    n, b, C, wn, al = 40, 6, 61.0, 1.0, 2.0
    cm = medium("c2", n)
    om, h, eta = O.problem_params(n, b, wn, al)
    Aref = O.build_A_matrix(b, C, eta, om, h, n, cm)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    A.krylov_mode("one")
    xr, infor, histr, _ = O.gmres_reference(Aref, f, M=O.jacobi_preconditioner(Aref), rtol=1e-4,
                                            restart=10, maxiter=400)
    x, info, hist = H.gmres(A, f, rtol=1e-4, restart=10, maxiter=400, M="jacobi",
                            callback=lambda r: None, callback_type='legacy', return_history=True)
    assert info == infor == 0 and len(hist) == len(histr)
    assert np.max(np.abs(hist - histr) / histr) < TOL
    assert relerr(x, xr) < TOL
    ref = []
    x3, info3 = scipy.sparse.linalg.gmres(Aref, f, rtol=1e-5, restart=10, maxiter=8,
                                          M=O.jacobi_preconditioner(Aref),
                                          callback=ref.append, callback_type="pr_norm")
    got = []
    x4, info4 = H.gmres(A, f, rtol=1e-5, restart=10, maxiter=8, M="jacobi", callback=got.append,
                        callback_type="pr_norm")
    assert info4 == info3 and len(got) == len(ref)
    assert np.max(np.abs(np.array(got) - np.array(ref)) / np.array(ref)) < TOL
    x0 = 1e-3 * rand_complex(n * n, 9)
    xr0, infor0, histr0, _ = O.gmres_reference(Aref, f, rtol=1e-3, restart=20, maxiter=60,
                                               x0=x0.copy())
    x5, info5, hist5 = H.gmres(A, f, x0=x0, rtol=1e-3, restart=20, maxiter=60,
                               callback=lambda r: None, callback_type='legacy',
                               return_history=True)
    assert info5 == infor0 and len(hist5) == len(histr0)
    assert np.max(np.abs(hist5 - histr0) / histr0) < TOL
    assert relerr(x5, xr0) < TOL


def test_one_allreduce_exact_solution_breakdown(ctx):
    """a right-hand side that is an eigenvector-like image (b = A e_p: the Krylov space closes
    at once for M = None on a 1x1-dominant system) must end with scipy's breakdown semantics"""
    import scipy.sparse.linalg
    n = 24
    om, h, eta = O.problem_params(n, 6, 2.0, 2.0)
    cm = medium("const", n)
    Aref = O.build_A_matrix(6, 61.0, eta, om, h, n, cm)
    A = H.build_A_matrix(6, 61.0, eta, om, h, n, cm, context=ctx)
    d = Aref.diagonal()
    f = d.copy()  # Jacobi-preconditioned system: M f = ones, M A ones = ... (closes quickly)
    A.krylov_mode("one")
    x, info = H.gmres(A, f, rtol=1e-10, restart=20, maxiter=3, M="jacobi")
    xr, infor = scipy.sparse.linalg.gmres(Aref, f, rtol=1e-10, restart=20, maxiter=3,
                                          M=O.jacobi_preconditioner(Aref))
    assert info == infor
    assert relerr(x, xr) < 1e-8


# ------------------------------------------- one pass over the basis (krylov mode "fused")
@pytest.mark.parametrize("name", ["gmres_n128_none.npz", "gmres_n128_jacobi.npz",
                                  "gmres_n64_c1_none.npz"])
def test_fused_pass_matches_reference_golden(ctx, name):
    """mode 3 (fused_iter_kernel: update, next M A and projections in one pass) against the
    reference's own histories -- partial strips (n < 256), one band per strip edge"""
    z = load_golden(name)
    n = int(z["n"])
    om = complex(z["omega"])
    cm = medium(str(z["medium"]), n)
    A = H.build_A_matrix(int(z["b"]), float(z["C"]), float(z["eta"]), om, float(z["h"]), n, cm,
                         context=ctx)
    A.krylov_mode("fused")
    A.small_cycle("off")
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    M = "jacobi" if str(z["precond"]) == "jacobi" else None
    hist = []
    x, info = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=int(z["K"]), M=M,
                      callback=hist.append, callback_type='legacy')
    hist = np.array(hist)
    assert A.last_solve_path() == "one-pass"
    assert info == int(z["info"]) and len(hist) == int(z["niter"])
    assert np.max(np.abs(hist - z["history"]) / z["history"]) < TOL
    assert relerr(x, z["x"]) < TOL


@pytest.mark.parametrize("n,kind,precond", [(300, "c1", "jacobi"), (513, "marmousi", None),
                                            (1100, "const", "jacobi"), (257, "c2", None),
                                            (300, "marmousi", "sl"), (770, "c1", "sl")])
@pytest.mark.parametrize("restart,K", [(20, 12), (7, 16), (1, 4), (21, 21)])
def test_fused_pass_matches_lagged(ctx, n, kind, precond, restart, K):
    """the one-pass iteration against the lagged one it fuses (same arithmetic but the inner
    products' summation order): ragged strips and bands, several restart cycles, legacy
    maxiter inside a cycle and at its edge, restart 1 (no fused pass at all: only the tail
    update) and the largest fused restart (21: K = 20 in the last pass)"""
    om, h, eta = O.problem_params(n, 12, n / 40.0, 2.0)
    cm = medium(kind, n) if kind != "marmousi" else H.marmousi_like_c_mat(n)
    A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm, context=ctx)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    if precond == "sl":  # (the two-sweep shifted Laplace: fused_sl_iter_kernel)
        precond = H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7)
    out = {}
    for mode in ("one", "fused"):
        A.krylov_mode(mode)
        hist = []
        x, info = H.gmres(A, f, rtol=1e-12, restart=restart, maxiter=K, M=precond,
                          callback=hist.append, callback_type='legacy')
        out[mode] = (x, info, np.array(hist), A.last_solve_path())
    (x1, i1, h1, p1), (x2, i2, h2, p2) = out["one"], out["fused"]
    assert p2 == "one-pass" and p1 != "one-pass"
    assert i1 == i2 and len(h1) == len(h2) == K
    # the first iterations to rounding; later ones within the parity contract (these stagnating
    # runs amplify a rounding difference ~100x per iteration past the tenth, as two scipy runs
    # on perturbed data do: DESIGN 6 'Where history parity is defined at all')
    k = min(K, 8)
    assert np.max(np.abs(h1[:k] - h2[:k]) / h1[:k]) < 1e-10
    assert np.max(np.abs(h1 - h2) / h1) < TOL
    assert relerr(x2, x1) < TOL


def test_fused_pass_is_the_single_rank_default(ctx):
    """mode auto on one rank picks the one-pass iteration where it applies (n >= 1024, M none /
    Jacobi / the two-sweep shifted Laplace, restart <= 21) and the regular cycle elsewhere
    (restart 30, three sweeps, n < 1024); mode "two" forces the regular cycle"""
    n = 1024
    om, h, eta = O.problem_params(n, 12, 64.0, 2.0)
    A = H.build_A_matrix(12, 81.0, eta, om, h, n, H.constant_c_mat(n), context=ctx)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    H.gmres(A, f, rtol=1e-12, restart=20, maxiter=5, M="jacobi")
    assert A.last_solve_path() == "one-pass"
    H.gmres(A, f, rtol=1e-12, restart=30, maxiter=5, M="jacobi")
    assert A.last_solve_path() == "regular"
    H.gmres(A, f, rtol=1e-12, restart=20, maxiter=3, M=H.ShiftedLaplace(A))
    assert A.last_solve_path() == "one-pass"
    H.gmres(A, f, rtol=1e-12, restart=20, maxiter=3, M=H.ShiftedLaplace(A, sweeps=3))
    assert A.last_solve_path() == "regular"
    A.krylov_mode("two")
    H.gmres(A, f, rtol=1e-12, restart=20, maxiter=3, M=H.ShiftedLaplace(A))
    assert A.last_solve_path() == "regular"
    A.krylov_mode("auto")
    n2 = 600
    om, h, eta = O.problem_params(n2, 12, 30.0, 2.0)
    B = H.build_A_matrix(12, 81.0, eta, om, h, n2, H.constant_c_mat(n2), context=ctx)
    H.gmres(B, O.init_f1_mat(.5, .125, om, n2).ravel(), rtol=1e-12, restart=20, maxiter=3,
            M=H.ShiftedLaplace(B))
    assert B.last_solve_path() == "regular"


_KEEP_CHILD = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import helmholtz_preconditioner_amd as H
n, kind, out = int(sys.argv[2]), sys.argv[3], sys.argv[4]
om, h, eta = H.problem_params(n, 12, n / 40.0, 2.0)
cm = H.marmousi_like_c_mat(n) if kind == "marmousi" else H.init_c1_mat(.5, .5, n)
A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm)
A.krylov_mode("fused")
f = H.init_f1_mat(.5, .125, om, n).ravel()
hist = []
x, info = H.gmres(A, f, rtol=1e-12, restart=21, maxiter=25, M="jacobi", callback=hist.append,
                  callback_type="legacy")
assert A.last_solve_path() == "one-pass"
np.savez(out, x=x, hist=np.array(hist), knobs=str(H.knobs()))
'''


@pytest.mark.parametrize("n,kind", [(300, "c1"), (1100, "marmousi")])
def test_fused_pass_lds_kept_basis_is_bit_identical(tmp_path, n, kind):
    """HH_FUSED_KEEP (read once per process, knobs.cpp): the projections' re-read of the first
    17 basis vectors from the pass's own one-row LDS copy (the default) instead of the memory
    system (0) reads the same values in the same order -- histories and fields bit-identical
    (K up to 20: the kept and re-read vectors mixed in one pass)"""
    import subprocess
    import sys
    out = []
    for keep in ("0", "17"):
        o = tmp_path / f"k{keep}.npz"
        subprocess.run([sys.executable, "-c", _KEEP_CHILD, ROOT, str(n), kind, str(o)],
                       env=dict(os.environ, HH_FUSED_KEEP=keep), check=True, timeout=240)
        out.append(np.load(o))
    # the child reports the knob it ran with (hh_knobs_json: only values off the default)
    assert "HH_FUSED_KEEP" in str(out[0]["knobs"]) and str(out[1]["knobs"]) == "{}"
    assert np.array_equal(out[1]["hist"], out[0]["hist"])
    assert np.array_equal(out[1]["x"], out[0]["x"])


def test_fused_keep_knob_refuses_unbuilt_counts():
    """HH_FUSED_KEEP selects between the two built forms (0: no LDS copy, 17: the default);
    any other count (round 3's A/B values 4, 8) is refused -- since round 6 when the knobs are
    read, at the first context -- instead of silently running 17"""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, sys.argv[1]); import helmholtz_preconditioner_amd as H; "
            "H.Context(device=0)")
    r = subprocess.run([sys.executable, "-c", code, ROOT], env=dict(os.environ, HH_FUSED_KEEP="4"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "HH_FUSED_KEEP=4" in r.stderr, r.stderr[-2000:]


@pytest.mark.parametrize("n,slabs", [(150, 2), (300, 3), (613, 4)])
@pytest.mark.parametrize("precond", [None, "jacobi", "sl"])
def test_fused_pass_virtual_slabs_match_single_slab(ctx, n, slabs, precond):
    """The one-pass iteration over several slabs of one rank (runtime.cpp run_fused: one launch
    per slab, the rows next to a slab boundary formed in place from the neighbouring slab,
    FROW_MEM -- two rows for the shifted Laplace) against the single slab: u and w are formed
    by the same arithmetic, only the projections' partial rows add in another order -- history
    and field (the dist tests' problem; restart 12, 26 iterations: three cycles)"""
    om, h, eta = H.problem_params(n, 12, 6.0, 2.0)
    cm = H.init_c1_mat(.5, .5, n)
    f = H.init_f1_mat(.5, .125, om, n).ravel()
    vctx = H.Context(device=0, virtual_slabs=slabs)
    out = []
    for c in (ctx, vctx):
        A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm, context=c)
        A.krylov_mode("fused")
        A.small_cycle("off")  # (n = 150, restart 12 would take the whole-cycle kernel)
        M = H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7) if precond == "sl" else precond
        x, info, hist = H.gmres(A, f, rtol=1e-3, restart=12, maxiter=26, M=M,
                                callback=lambda r: None, callback_type="legacy",
                                return_history=True)
        assert A.last_solve_path() == "one-pass"
        out.append((x, info, np.asarray(hist)))
        A.close()
    vctx.close()
    (x1, i1, h1), (x2, i2, h2) = out
    assert i1 == i2 and len(h1) == len(h2)
    # the first iterations to rounding (the reordered sums' last bits); later iterations
    # amplify that rounding (DESIGN 6 'Where history parity is defined at all'): the whole
    # history and the field within the parity contract.  Measured (tools/slab_drift.py,
    # profiles/r05/r05_slab_drift_cpu_613_jacobi.log): the numpy mirror of this very solve
    # (tests/dist_mirror.py gmres_dist_onepass), whose slab split changes NOTHING but the inner
    # products' summation order, drifts 1.0e-15 by iteration 5 and 1.5e-8 by iteration 10 at
    # n = 613 / 4 slabs / Jacobi (a stagnating run: presid 4e-7 throughout), and scipy itself
    # 6.9e-4 on f vs f (1 + 1e-15) -- the device's 1.35e-8 (round 4) is that amplification
    assert np.max(np.abs(h1[:5] - h2[:5]) / h1[:5]) < 1e-10
    assert np.max(np.abs(h1 - h2) / h1) < TOL
    assert relerr(x2, x1) < TOL


_CHILD = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import helmholtz_preconditioner_amd as H
n, kind, restart, K, out = int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
om, h, eta = H.problem_params(n, 12, n / 40.0, 2.0)
cm = H.marmousi_like_c_mat(n) if kind == "marmousi" else H.init_c1_mat(.5, .5, n)
A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm)
A.krylov_mode("fused")
f = H.init_f1_mat(.5, .125, om, n).ravel()
x, info, hist = H.gmres(A, f, rtol=1e-12, restart=restart, maxiter=K, M="jacobi",
                        callback=lambda r: None, callback_type="legacy", return_history=True)
assert A.last_solve_path() == "one-pass"
np.savez(out, x=x, info=info, hist=hist)
'''


@pytest.mark.parametrize("n,kind,restart,K", [(300, "c1", 20, 45), (1100, "marmousi", 7, 22),
                                              (257, "c1", 1, 5), (513, "c1", 21, 30)])
def test_fused_cycle_end_merge_matches_solve_and_xupdate(tmp_path, n, kind, restart, K):
    """The end of a full one-pass cycle in one pass (fused.hip cycle_end_kernel: the last
    update's norm, x += V a and V b from the same loads, then x += y_col V b) against the
    separate update, triangular solve and xupdate (HH_CYCLE_MERGE=0): the first cycle's history
    identical, x and the later cycles to rounding (x = x + V a + y_col V b instead of x + V y).
    Cycles that stop before their last column take the solve + xupdate either way (legacy
    maxiter inside a cycle: K = 45 / restart 20, 22 / 7)."""
    import subprocess
    import sys
    res = []
    for merge in ("1", "0"):
        out = tmp_path / f"m{merge}.npz"
        env = dict(os.environ, HH_CYCLE_MERGE=merge)
        subprocess.run([sys.executable, "-c", _CHILD, ROOT, str(n), kind, str(restart), str(K),
                        str(out)], env=env, check=True, timeout=240)
        res.append(np.load(out))
    a, b = res
    assert int(a["info"]) == int(b["info"]) and len(a["hist"]) == len(b["hist"]) == K
    c = min(restart, K)
    assert np.array_equal(a["hist"][:c], b["hist"][:c])
    assert np.max(np.abs(a["hist"] - b["hist"]) / b["hist"]) < 1e-9
    assert relerr(a["x"], b["x"]) < 1e-11



@pytest.mark.parametrize("n,kind,restart,K", [(300, "c1", 20, 45), (1100, "marmousi", 7, 22),
                                              (1024, "c1", 21, 25)])
def test_fused_lag_reduce_merge_bit_identical(tmp_path, n, kind, restart, K):
    """One rank: the partial-row reduce and the lag step in one launch (krylov.hip
    gmres_lag_red_kernel, reduce_kernel's 256-thread summation order played by 8 waves) against
    the two launches (HH_LAG_RED=0): history and x bit for bit."""
    import subprocess
    import sys
    res = []
    for merge in ("1", "0"):
        out = tmp_path / f"l{merge}.npz"
        env = dict(os.environ, HH_LAG_RED=merge)
        subprocess.run([sys.executable, "-c", _CHILD, ROOT, str(n), kind, str(restart), str(K),
                        str(out)], env=env, check=True, timeout=240)
        res.append(np.load(out))
    a, b = res
    assert int(a["info"]) == int(b["info"]) and len(a["hist"]) == len(b["hist"]) == K
    assert np.array_equal(a["hist"], b["hist"])
    assert np.array_equal(a["x"], b["x"])

_SLK_CHILD = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import helmholtz_preconditioner_amd as H
n, kind, slabs, restart, K, out = (int(sys.argv[2]), sys.argv[3], int(sys.argv[4]),
                                    int(sys.argv[5]), int(sys.argv[6]), sys.argv[7])
om, h, eta = H.problem_params(n, 12, n / 40.0, 2.0)
cm = H.marmousi_like_c_mat(n) if kind == "marmousi" else H.init_c1_mat(.5, .5, n)
ctx = H.Context(device=0, virtual_slabs=slabs)
A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm, context=ctx)
A.krylov_mode("fused")
A.small_cycle("off")
M = H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7)
f = H.init_f1_mat(.5, .125, om, n).ravel()
x, info, hist = H.gmres(A, f, rtol=1e-12, restart=restart, maxiter=K, M=M,
                        callback=lambda r: None, callback_type="legacy", return_history=True)
assert A.last_solve_path() == "one-pass"
np.savez(out, x=x, info=info, hist=hist)
'''


@pytest.mark.parametrize("n,kind,slabs", [(300, "c1", 1), (257, "marmousi", 3), (1024, "c1", 2)])
def test_sl_residual_one_pass_matches_three_launches(tmp_path, n, kind, slabs):
    """The shifted-Laplace residual v0 = M (b - A x) in one pass (sl_fused.hip sl2_res_kernel,
    with |r|^2 and |M r|^2) against the three launches (HH_SL_RES=0: r and z1, the second sweep,
    the norm): v0 is formed by the same per-point arithmetic (not compared directly here: the
    solve exposes only its history and x), the norms are summed in another order -- the
    histories agree to rounding at the start and within the parity contract after (stagnating
    runs amplify)."""
    import subprocess
    import sys
    res = []
    for fused in ("1", "0"):
        out = tmp_path / f"r{fused}.npz"
        env = dict(os.environ, HH_SL_RES=fused)
        subprocess.run([sys.executable, "-c", _SLK_CHILD, ROOT, str(n), kind, str(slabs), "20",
                        "25", str(out)], env=env, check=True, timeout=240)
        res.append(np.load(out))
    a, b = res
    assert int(a["info"]) == int(b["info"]) and len(a["hist"]) == len(b["hist"]) == 25
    assert np.max(np.abs(a["hist"][:3] - b["hist"][:3]) / b["hist"][:3]) < 1e-12
    assert np.max(np.abs(a["hist"] - b["hist"]) / b["hist"]) < TOL
    assert relerr(a["x"], b["x"]) < TOL


@pytest.mark.parametrize("n,kind,slabs,rows", [(300, "c1", 1, 16), (1100, "marmousi", 1, 32),
                                               (613, "marmousi", 3, 16), (257, "c1", 2, 8)])
def test_fused_sl_keep_kernel_bit_identical(tmp_path, n, kind, slabs, rows):
    """fused_slk.hip (the shifted-Laplace pass with its whole basis window on chip: a three-row
    LDS ring for 11 vectors, a four-slot register ring for the rest, one block per CU) against
    fused.hip fused_sl_iter_kernel (5 vectors kept, the rest re-read) on the same bands
    (HH_FUSED_ROWS = HH_SLK_ROWS): the same arithmetic in the same order, so histories and
    fields are bit-identical -- restart 21, 25 iterations (K = 1 .. 20: both rings, and a second
    cycle), ragged strips and bands, virtual slabs (rows formed in place across slabs)"""
    import subprocess
    import sys
    res = []
    for slk in ("0", "1"):
        out = tmp_path / f"slk{slk}.npz"
        env = dict(os.environ, HH_SLK=slk, HH_FUSED_ROWS=str(rows), HH_SLK_ROWS=str(rows))
        subprocess.run([sys.executable, "-c", _SLK_CHILD, ROOT, str(n), kind, str(slabs), "21",
                        "25", str(out)], env=env, check=True, timeout=240)
        res.append(np.load(out))
    a, b = res
    assert int(a["info"]) == int(b["info"]) and len(a["hist"]) == len(b["hist"]) == 25
    assert np.array_equal(a["hist"], b["hist"])
    assert np.array_equal(a["x"], b["x"])


_ALT_CHILD = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import helmholtz_preconditioner_amd as H
n, kind, pc, out = int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
om, h, eta = H.problem_params(n, 12, n / 40.0, 2.0)
cm = H.marmousi_like_c_mat(n) if kind == "marmousi" else H.init_c1_mat(.5, .5, n)
A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm)
A.krylov_mode("fused")
A.small_cycle("off")
f = H.init_f1_mat(.5, .125, om, n).ravel()
x, info, hist = H.gmres(A, f, rtol=1e-12, restart=20, maxiter=30, M=None if pc == "none" else pc,
                        callback=lambda r: None, callback_type="legacy", return_history=True)
assert A.last_solve_path() == "one-pass"
np.savez(out, x=x, info=info, hist=hist)
'''


@pytest.mark.parametrize("n,kind,pc", [(1024, "c1", "jacobi"), (613, "marmousi", "none")])
def test_fused_pass_alternating_march_matches(tmp_path, n, kind, pc):
    """HH_FUSED_ALT=1 (fused_iter_kernel's odd bands march downwards, so a band's re-formed halo
    rows are read while their owner reads them) against the all-upward march: per point the
    same arithmetic, only the order of a band's rows in its partial row differs -- the first
    iterations to rounding, the 30-iteration history and the field within the parity
    contract."""
    import subprocess
    import sys
    res = []
    for alt in ("0", "1"):
        out = tmp_path / f"alt{alt}.npz"
        env = dict(os.environ, HH_FUSED_ALT=alt)
        subprocess.run([sys.executable, "-c", _ALT_CHILD, ROOT, str(n), kind, pc, str(out)],
                       env=env, check=True, timeout=240)
        res.append(np.load(out))
    a, b = res
    assert int(a["info"]) == int(b["info"]) and len(a["hist"]) == len(b["hist"]) == 30
    assert np.max(np.abs(a["hist"][:5] - b["hist"][:5]) / a["hist"][:5]) < 1e-10
    assert np.max(np.abs(a["hist"] - b["hist"]) / a["hist"]) < TOL
    assert relerr(b["x"], a["x"]) < TOL


@pytest.mark.parametrize("n,kind,slabs", [(300, "c1", 1), (257, "marmousi", 3), (1100, "marmousi", 1),
                                          (613, "c1", 2)])
def test_fused_sl_overlapping_strip_kernel_matches(tmp_path, n, kind, slabs):
    """fused_slv.hip (the shifted-Laplace pass in the standalone fused M A's shape: overlapping
    252-column strips, no edge waves; HH_SLV = the largest K it takes) against the edge-wave
    kernels (HH_SLV=0: fused_sl_iter_kernel / fused_slk_kernel) on the same problem: the same
    operator and preconditioner arithmetic, only the strip-edge columns' u_K (k order here, a
    shuffle tree there) and the projections' summation order differ -- the first iterations to
    rounding, the 25-iteration history (K = 1 .. 20: both kernels in one cycle, then a second
    cycle) and the field within the parity contract; ragged strips, virtual slabs."""
    import subprocess
    import sys
    res = []
    for slv in ("0", "6"):
        out = tmp_path / f"slv{slv}.npz"
        env = dict(os.environ, HH_SLV=slv)
        subprocess.run([sys.executable, "-c", _SLK_CHILD, ROOT, str(n), kind, str(slabs), "21",
                        "25", str(out)], env=env, check=True, timeout=240)
        res.append(np.load(out))
    a, b = res
    assert int(a["info"]) == int(b["info"]) and len(a["hist"]) == len(b["hist"]) == 25
    assert np.max(np.abs(a["hist"][:5] - b["hist"][:5]) / a["hist"][:5]) < 1e-10
    assert np.max(np.abs(a["hist"] - b["hist"]) / a["hist"]) < TOL
    assert relerr(b["x"], a["x"]) < TOL


# Grids: 130^2 (17 blocks: fewer than the 64 residue classes), 1024^2 (config 2's: 512 blocks,
# 8 a class; a stagnating solve whose field moves 1e-6 under any reordering -- bit-identical
# here), 2500^2 (3130 blocks: 49 a class, four rounds of row loads), ragged strips, restarts
# and the shifted-Laplace passes (fused_slv / fused_slk).
@pytest.mark.parametrize("n,kind,restart,K,pc", [(300, "c1", 20, 45, "jacobi"),
                                                 (1100, "marmousi", 7, 22, "jacobi"),
                                                 (1024, "c1", 20, 30, "jacobi"),
                                                 (613, "marmousi", 20, 30, "none"),
                                                 (257, "c1", 1, 5, "jacobi"),
                                                 (130, "c1", 20, 25, "jacobi"),
                                                 (2500, "marmousi", 20, 6, "jacobi"),
                                                 (1100, "marmousi", 21, 25, "sl")])
def test_in_pass_column_matches_separate_launches(tmp_path, n, kind, restart, K, pc):
    """HH_LAG_RED=2 (the default on one slab of one rank): the one-pass kernels' own blocks
    reduce their partial rows -- the blocks of each residue class mod 64 in block order, then the
    classes by reduce_kernel's shuffle tree -- and the last one runs the lag step
    (hh_fused.hpp pass_fold), instead of the reduce + lag launches (HH_LAG_RED=0) or the merged
    launch (1): reduce_kernel's summation order exactly, so histories and fields are bit for bit
    the launches' whatever order the blocks arrive in."""
    import subprocess
    import sys
    code = _ALT_CHILD.replace('restart=20, maxiter=30', f'restart={restart}, maxiter={K}')
    res = []
    for mode in ("0", "2", "1"):
        out = tmp_path / f"m{mode}.npz"
        env = dict(os.environ, HH_LAG_RED=mode)
        args = ([_SLK_CHILD, ROOT, str(n), kind, "1", str(restart), str(K), str(out)] if pc == "sl"
                else [code, ROOT, str(n), kind, pc, str(out)])
        subprocess.run([sys.executable, "-c"] + args, env=env, check=True, timeout=240)
        res.append(np.load(out))
    a, b, c = res
    assert int(a["info"]) == int(b["info"]) and len(a["hist"]) == len(b["hist"]) == K
    for o in (b, c):
        assert np.array_equal(o["hist"], a["hist"]) and np.array_equal(o["x"], a["x"])
