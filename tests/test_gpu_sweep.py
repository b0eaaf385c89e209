"""GPU tier, SURVEY row F1: the sweeping moving-PML preconditioner (algo2_3 / algo2_4,
code.py:345-385) on the device (csrc/sweep.hip, block Thomas instead of SuperLU).

* as-is (the reference's run, quirks Q1/Q2) against golden vectors produced by the
  reference's own algo2_4 (tests/golden/sweep_*.npz): 1e-10 relative;
* corrected (Alg. 2.4) against the oracle's SuperLU restatement: apply 1e-10, GMRES
  history / field 1e-6 (contract).
"""
import os

import numpy as np
import pytest

import helmholtz_preconditioner_amd as H
from conftest import load_golden, medium, rand_complex
from oracle import helmholtz_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = H.Context(device=0)
    H.set_default_context(c)
    yield c
    H.set_default_context(None)


def relerr(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


def _case(z, ctx):
    n, b = int(z["n"]), int(z["b"])
    om, C, h, eta = complex(z["omega"]), float(z["C"]), float(z["h"]), float(z["eta"])
    cm = medium(str(z["medium"]), n)
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    return A, (b, C, eta, om, h, n, cm)


@pytest.mark.parametrize("name", ["sweep_n48_c1.npz", "sweep_n37_c2.npz"])
def test_sweep_as_is_matches_reference(ctx, name):
    z = load_golden(name)
    A, (b, C, eta, om, h, n, cm) = _case(z, ctx)
    M = H.Sweeping(A, reference=True)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    assert relerr(M @ f, z["u_f"]) < 1e-10
    assert relerr(M @ rand_complex(n * n, 3), z["u_x"]) < 1e-10


@pytest.mark.parametrize("name", ["sweep_n48_c1.npz", "sweep_n37_c2.npz"])
def test_sweep_corrected_matches_oracle(ctx, name):
    z = load_golden(name)
    A, (b, C, eta, om, h, n, cm) = _case(z, ctx)
    st = O.SweepState(b, C, eta, om, h, n, cm)
    M = H.Sweeping(A)
    for seed in (0, 1):
        x = rand_complex(n * n, seed)
        assert relerr(M @ x, st.apply(x, corrected=True)) < 1e-10


@pytest.mark.parametrize("n,b,kind", [(96, 12, "c1"), (130, 8, "const"), (200, 16, "c2"),
                                      (61, 5, "c1")])
def test_sweep_sizes_vs_oracle(ctx, n, b, kind):
    om, h, eta = O.problem_params(n, b, 5.0, 2.0)
    cm = medium(kind, n)
    A = H.build_A_matrix(b, 81.0, eta, om, h, n, cm, context=ctx)
    st = O.SweepState(b, 81.0, eta, om, h, n, cm)
    x = rand_complex(n * n, n)
    assert relerr(H.Sweeping(A) @ x, st.apply(x, corrected=True)) < 1e-10
    assert relerr(H.Sweeping(A, reference=True) @ x, st.apply(x)) < 1e-10


@pytest.mark.parametrize("name", ["sweep_n48_c1.npz", "sweep_n37_c2.npz"])
def test_gmres_corrected_sweeping_vs_oracle(ctx, name):
    z = load_golden(name)
    A, (b, C, eta, om, h, n, cm) = _case(z, ctx)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    Aref = O.build_A_matrix(b, C, eta, om, h, n, cm)
    Mref, _ = O.sweeping_preconditioner(b, C, eta, om, h, n, cm, corrected=True)
    xr, infor, histr, relr = O.gmres_reference(Aref, f, M=Mref, rtol=1e-3, restart=20, maxiter=200)
    x, info, hist = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=200, M=H.Sweeping(A),
                            callback=lambda r: None, callback_type="legacy", return_history=True)
    assert info == infor == 0 and len(hist) == len(histr)
    assert np.max(np.abs(hist - histr) / histr) < 1e-6
    assert relerr(x, xr) < 1e-6


@pytest.mark.parametrize("name", ["sweep_n48_c1.npz", "sweep_n37_c2.npz"])
def test_gmres_reference_run_as_is(ctx, name):
    """the reference's own solve (code.py:516 with M of code.py:510): M is a constant map, so
    every cycle's Krylov space is one-dimensional and GMRES sits ON scipy's breakdown test
    h1 <= eps*h0 (iterative.py:767) -- h1 is the rounding residue of c - <v0,c> v0, so how
    many cycles run before the test fires (1..3 here) is decided by rounding noise, not by
    the algorithm.  What is reproducible: info == maxiter (not converged) and a ~0 history."""
    z = load_golden(name)
    A, (b, C, eta, om, h, n, cm) = _case(z, ctx)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    x, info, hist = H.gmres(A, f, rtol=1e-3, M=H.Sweeping(A, reference=True),
                            callback=lambda r: None, callback_type="legacy", return_history=True)
    assert info == int(z["gmres_info"])
    assert 1 <= len(hist) <= 3 and 1 <= len(z["gmres_hist"]) <= 3
    assert np.all(np.abs(hist) < 1e-12)  # the reference's presid history is ~0 (breakdown)


# ---------------------------------------------------------------- dense-transfer form
@pytest.mark.parametrize("n,b,kind", [(96, 12, "c1"), (130, 8, "const"), (61, 5, "c1"),
                                      (13, 12, "c2"), (200, 16, "c2"), (300, 12, "c1")])
def test_sweep_dense_matches_thomas_and_oracle(ctx, n, b, kind):
    om, h, eta = O.problem_params(n, b, 5.0, 2.0)
    cm = medium(kind, n)
    A = H.build_A_matrix(b, 81.0, eta, om, h, n, cm, context=ctx)
    x = rand_complex(n * n, n + 1)
    st = O.SweepState(b, 81.0, eta, om, h, n, cm) if n <= 200 else None
    for reference in (False, True):
        Md = H.Sweeping(A, reference=reference, form="dense")
        yd = Md @ x
        assert Md.dense
        Mt = H.Sweeping(A, reference=reference, form="thomas")
        yt = Mt @ x
        assert not Mt.dense
        assert relerr(yd, yt) < 1e-10
        if st is not None:
            assert relerr(yd, st.apply(x, corrected=not reference)) < 1e-10


def test_sweep_dense_large_rows(ctx):
    """n > 1024: the 32-chunk GEMV rows and several setup chunks per system."""
    n, b = 1100, 12
    om, h, eta = O.problem_params(n, b, 40.0, 2.0)
    A = H.build_A_matrix(b, 81.0, eta, om, h, n, O.init_c1_mat(.5, .5, n), context=ctx)
    x = rand_complex(n * n, 11)
    yd = H.Sweeping(A, form="dense") @ x
    yt = H.Sweeping(A, form="thomas") @ x
    assert relerr(yd, yt) < 1e-9


@pytest.mark.parametrize("name", ["sweep_n48_c1.npz", "sweep_n37_c2.npz"])
def test_sweep_dense_as_is_matches_reference_golden(ctx, name):
    z = load_golden(name)
    A, (b, C, eta, om, h, n, cm) = _case(z, ctx)
    M = H.Sweeping(A, reference=True, form="dense")
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    assert relerr(M @ f, z["u_f"]) < 1e-10
    assert relerr(M @ rand_complex(n * n, 3), z["u_x"]) < 1e-10


def test_gmres_dense_sweeping_vs_oracle(ctx):
    z = load_golden("sweep_n48_c1.npz")
    A, (b, C, eta, om, h, n, cm) = _case(z, ctx)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    Aref = O.build_A_matrix(b, C, eta, om, h, n, cm)
    Mref, _ = O.sweeping_preconditioner(b, C, eta, om, h, n, cm, corrected=True)
    xr, infor, histr, _ = O.gmres_reference(Aref, f, M=Mref, rtol=1e-3, restart=20, maxiter=200)
    x, info, hist = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=200,
                            M=H.Sweeping(A, form="dense"), callback=lambda r: None,
                            callback_type="legacy", return_history=True)
    assert info == infor == 0 and len(hist) == len(histr)
    assert np.max(np.abs(hist - histr) / histr) < 1e-6
    assert relerr(x, xr) < 1e-6


@pytest.mark.parametrize("n,b,kind", [(13, 12, "c2"), (96, 12, "c1"), (300, 12, "c1"),
                                      (1023, 12, "c1")])
def test_sweep_persistent_chain_bit_identical_to_launches(ctx, n, b, kind):
    """the dense apply as ONE persistent launch (form "dense", n <= 1024) against one launch per
    GEMV (form "dense-launches"): same lane partition, FMA order and DPP reduction -- the same
    bits, both modes, also inside a GMRES cycle (its stop flag ends the chain early)"""
    om, h, eta = O.problem_params(n, b, 5.0, 2.0)
    A = H.build_A_matrix(b, 81.0, eta, om, h, n, medium(kind, n), context=ctx)
    x = rand_complex(n * n, n + 7)
    for reference in (False, True):
        yc = H.Sweeping(A, reference=reference, form="dense") @ x
        yl = H.Sweeping(A, reference=reference, form="dense-launches") @ x
        assert np.array_equal(yc, yl)
    if n <= 300:
        f = O.init_f1_mat(.5, .125, om, n).ravel()
        out = []
        for form in ("dense", "dense-launches"):
            out.append(H.gmres(A, f, rtol=1e-3, restart=20, maxiter=60,
                               M=H.Sweeping(A, form=form), callback=lambda r: None,
                               callback_type="legacy", return_history=True))
        (x1, i1, h1), (x2, i2, h2) = out
        assert i1 == i2 and np.array_equal(h1, h2) and np.array_equal(x1, x2)


# ------------------------------------------------------- partitioned block-Thomas solves
@pytest.mark.parametrize("name", ["sweep_n48_c1.npz", "sweep_n37_c2.npz"])
@pytest.mark.parametrize("form", ["thomas", "thomas-sequential"])
def test_sweep_thomas_as_is_matches_reference_golden(ctx, name, form):
    """the solve forms (n >= 32: "thomas" partitions every forward / backward-sweep solve over
    16 column chunks) against the reference's own algo2_4 outputs"""
    z = load_golden(name)
    A, (b, C, eta, om, h, n, cm) = _case(z, ctx)
    M = H.Sweeping(A, reference=True, form=form)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    assert relerr(M @ f, z["u_f"]) < 1e-10
    assert M.partitioned == (form == "thomas")
    assert relerr(M @ rand_complex(n * n, 3), z["u_x"]) < 1e-10


@pytest.mark.parametrize("n,b,kind,wgs", [(32, 5, "c1", 0), (33, 12, "c2", 0), (61, 5, "c1", 0),
                                          (96, 12, "c1", 3), (130, 8, "const", 4),
                                          (200, 16, "c2", 0), (257, 3, "c1", 0),
                                          (257, 3, "c1", 8), (331, 12, "c2", 0),
                                          (331, 12, "c2", 2), (700, 12, "c1", 0),
                                          (700, 16, "c1", 0), (700, 16, "c1", 21),
                                          (1300, 12, "c2", 40)])
def test_sweep_partitioned_vs_sequential_and_oracle(ctx, n, b, kind, wgs):
    """ragged chunks (n not a multiple of 8), every block size B = 4, 8, 12, 16, both sweeps,
    one workgroup and several (wgs 0: by n -- 700: 21 workgroups, every solve's carries cross
    workgroups through the granule exchange; 21 at B = 16 and 40 at B = 12: more upstream
    workgroups than the grid maps each half-wave holds ahead of the exchange, so the rest are
    loaded after it)"""
    om, h, eta = O.problem_params(n, b, 5.0, 2.0)
    cm = medium(kind, n)
    A = H.build_A_matrix(b, 81.0, eta, om, h, n, cm, context=ctx)
    x = rand_complex(n * n, n + 3)
    st = O.SweepState(b, 81.0, eta, om, h, n, cm) if n <= 200 else None
    want = min(wgs if wgs else n // 32, 64, n // 32) or 1
    for reference in (False, True):
        Mp = H.Sweeping(A, reference=reference, form="thomas", workgroups=wgs)
        yp = Mp @ x
        assert Mp.partitioned and not Mp.dense
        assert Mp.workgroups == max(want, 1)
        Ms = H.Sweeping(A, reference=reference, form="thomas-sequential")
        ys = Ms @ x
        assert not Ms.partitioned and not Ms.dense
        assert relerr(yp, ys) < 1e-10
        if st is not None:
            assert relerr(yp, st.apply(x, corrected=not reference)) < 1e-10


def test_gmres_partitioned_sweeping_vs_oracle(ctx):
    z = load_golden("sweep_n48_c1.npz")
    A, (b, C, eta, om, h, n, cm) = _case(z, ctx)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    Aref = O.build_A_matrix(b, C, eta, om, h, n, cm)
    Mref, _ = O.sweeping_preconditioner(b, C, eta, om, h, n, cm, corrected=True)
    xr, infor, histr, _ = O.gmres_reference(Aref, f, M=Mref, rtol=1e-3, restart=20, maxiter=200)
    x, info, hist = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=200,
                            M=H.Sweeping(A, form="thomas"), callback=lambda r: None,
                            callback_type="legacy", return_history=True)
    assert info == infor == 0 and len(hist) == len(histr)
    assert np.max(np.abs(hist - histr) / histr) < 1e-6
    assert relerr(x, xr) < 1e-6


def test_sweep_partitioned_large_linearity(ctx):
    """n = 4095 (beyond the dense form's n <= 2048): the partitioned corrected-sweep apply runs
    and is linear to rounding, M (x + 2i y) = M x + 2i M y (no oracle at this size)"""
    n, b = 4095, 12
    om, h, eta = O.problem_params(n, b, 100.0, 2.0)
    A = H.build_A_matrix(b, 81.0, eta, om, h, n, O.init_c1_mat(.5, .5, n), context=ctx)
    M = H.Sweeping(A, form="auto")
    M.configure()
    assert M.partitioned
    x, y = rand_complex(n * n, 1), rand_complex(n * n, 2)
    mx, my, mxy = M @ x, M @ y, M @ (x + 2j * y)
    assert np.all(np.isfinite(mxy))
    assert relerr(mxy, mx + 2j * my) < 1e-10


def test_sweep_partitioned_workgroups_agree_with_dense(ctx):
    """n = 1023 (the dense form's largest persistent-chain size): the partitioned apply over
    1, 4, 15 and 31 (auto) workgroups agrees with the dense transfer form to rounding"""
    n, b = 1023, 12
    om, h, eta = O.problem_params(n, b, 128.0, 2.0)
    A = H.build_A_matrix(b, 100.0, eta, om, h, n, O.init_c1_mat(.5, .5, n), context=ctx)
    x = rand_complex(n * n, 11)
    yd = H.Sweeping(A, form="dense") @ x
    for wgs, want in ((1, 1), (4, 4), (15, 15), (0, 31)):
        M = H.Sweeping(A, form="thomas", workgroups=wgs)
        y = M @ x
        assert M.partitioned and M.workgroups == want
        assert relerr(y, yd) < 1e-10


_PLAIN_LAUNCH = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import helmholtz_preconditioner_amd as H
from helmholtz_preconditioner_amd import _ffi
out = sys.argv[2]
res = {}
for n, form in ((300, "thomas"), (255, "dense")):
    om, h, eta = H.problem_params(n, 12, n / 8 + 1, 2.0)
    cm, f = H.init_c1_f1(om, n)
    A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm)
    M = H.Sweeping(A, form=form, workgroups=4 if form == "thomas" else 0)
    M.configure()
    x, y = A.vector(f.ravel()), A.vector()
    A.apply_device(x, y, _ffi.HH_APPLY_PREC)
    res[form] = y.download()
    res[form + "_grid"] = np.array([M.partitioned or M.dense, M.workgroups])
    x.close(); y.close(); A.close()
np.savez(out, **res)
'''


def test_sweep_plain_launch_matches_cooperative(tmp_path):
    """HH_SWEEP_COOP=0 (the grid-wide sweeps -- partitioned block-Thomas over 4 workgroups, the
    dense form's persistent chain -- as plain launches; profiling runs use it) gives
    bit-identical applies: only the launch API differs, the kernels and their bounded grid
    waits are the same.  Child processes: the switch is read once per process."""
    import subprocess
    import sys
    from conftest import ROOT
    outs = []
    for coop in ("1", "0"):
        out = tmp_path / f"c{coop}.npz"
        subprocess.run([sys.executable, "-c", _PLAIN_LAUNCH, ROOT, str(out)], check=True,
                       timeout=240, env=dict(os.environ, HH_SWEEP_COOP=coop))
        outs.append(np.load(out))
    a, b = outs
    assert int(a["thomas_grid"][1]) == 4
    for k in ("thomas", "dense"):
        np.testing.assert_array_equal(a[k], b[k])
