"""CPU tier: pin the oracle (oracle/helmholtz_oracle.py) to the reference's own outputs.

The golden vectors in tests/golden/ were produced by importing the reference
code.py itself (tests/golden/make_golden.py).  Tolerances: coefficients and SpMV
1e-13 relative (the oracle restates the same float64 formulas; differences are
ulp-level complex-division rounding), GMRES residual histories 1e-8 relative.
"""
import numpy as np
import pytest

from conftest import load_golden, medium, rand_complex
from oracle import helmholtz_oracle as O
import helmholtz_preconditioner_amd.media as media  # host-only module (no GPU needed)

COEF = ["coef_n16_c1.npz", "coef_n33_c2.npz", "coef_n64_const.npz", "coef_n64_c1.npz"]


def _A(z, cm=None):
    n = int(z["n"])
    if cm is None:
        cm = medium(str(z["medium"]), n)
    return O.build_A_matrix(int(z["b"]), float(z["C"]), float(z["eta"]), complex(z["omega"]),
                            float(z["h"]), n, cm)


def test_inputs_match_reference():
    z = load_golden("inputs.npz")
    n, om = int(z["n"]), complex(z["omega"])
    for mod in (O, media):
        np.testing.assert_array_equal(mod.init_c1_mat(.5, .5, n), z["c1"])
        np.testing.assert_array_equal(mod.init_c1_mat(.3, .6, n), z["c1_off"])
        np.testing.assert_array_equal(mod.init_c2_mat(n), z["c2"])
        np.testing.assert_allclose(mod.init_f1_mat(.5, .125, om, n), z["f1"], rtol=1e-14, atol=0)
        np.testing.assert_allclose(mod.init_f2_mat(.125, .125, 1 / 2 ** .5, 1 / 2 ** .5, om, n),
                                   z["f2"], rtol=1e-13, atol=1e-300)


@pytest.mark.parametrize("n,j0,j1", [(33, 0, 33), (150, 37, 101), (257, 250, 257)])
def test_f1_rows_are_the_slab_of_init_f1_mat(n, j0, j1):
    """A rank's rows of the source (media.init_f1_rows: bench.py and the multi-rank workers,
    which must not form the whole n x n grid at 16384^2) are bit for bit rows j0 .. j1 of
    init_f1_mat, the golden-pinned reference input."""
    om = complex(n / 3.0, 0.25)
    np.testing.assert_array_equal(media.init_f1_rows(.5, .125, om, n, j0, j1),
                                  media.init_f1_mat(.5, .125, om, n)[j0:j1])


@pytest.mark.parametrize("name", COEF)
def test_csr_matches_reference(name):
    z = load_golden(name)
    A = _A(z)
    assert A.nnz == len(z["data"])
    np.testing.assert_array_equal(A.indptr, z["indptr"])
    np.testing.assert_array_equal(A.indices, z["indices"])
    rel = np.abs(A.data - z["data"]) / np.abs(z["data"])
    assert rel.max() < 1e-13


def test_shifted_operator_matches_reference():
    z = load_golden("shift_n64.npz")
    n = int(z["n"])
    A = _A(z, O.init_c1_mat(.5, .5, n) / np.sqrt(1 + 1j * float(z["beta"])))
    np.testing.assert_array_equal(A.indices, z["indices"])
    assert (np.abs(A.data - z["data"]) / np.abs(z["data"])).max() < 1e-13


@pytest.mark.parametrize("name", ["spmv_n128_const.npz", "spmv_n257_c1.npz"])
def test_spmv_matches_reference(name):
    z = load_golden(name)
    n = int(z["n"])
    x = rand_complex(n * n, 0)
    np.testing.assert_array_equal(x[:64], z["x_head"])  # generator unchanged
    y = _A(z) @ x
    assert np.linalg.norm(y - z["y"]) / np.linalg.norm(z["y"]) < 1e-14


@pytest.mark.parametrize("name", ["gmres_n128_none.npz", "gmres_n128_jacobi.npz",
                                  "gmres_n64_c1_none.npz"])
def test_gmres_matches_reference(name):
    z = load_golden(name)
    n = int(z["n"])
    A = _A(z)
    f = O.init_f1_mat(.5, .125, complex(z["omega"]), n).ravel()
    M = O.jacobi_preconditioner(A) if str(z["precond"]) == "jacobi" else None
    x, info, hist, relres = O.gmres_reference(A, f, M=M, rtol=1e-3, restart=20, maxiter=int(z["K"]))
    assert info == int(z["info"])
    assert len(hist) == int(z["niter"])
    assert np.max(np.abs(hist - z["history"]) / z["history"]) < 1e-8
    assert np.linalg.norm(x - z["x"]) / np.linalg.norm(z["x"]) < 1e-8
    assert abs(relres - float(z["relres"])) / float(z["relres"]) < 1e-8


def test_operator_is_complex_symmetric():
    z = load_golden("coef_n33_c2.npz")
    A = _A(z)
    assert abs(A - A.T).max() == 0.0  # A - A^T == 0 bitwise


@pytest.mark.parametrize("bounds", [[(0, 17), (17, 33)], [(0, 5), (5, 6), (6, 33)],
                                    [(0, 7), (7, 14), (14, 21), (21, 28), (28, 33)]])
def test_slab_emulator_equals_global_apply(bounds):
    z = load_golden("coef_n33_c2.npz")
    n = int(z["n"])
    cm = medium("c2", n)
    x = rand_complex(n * n, 3)
    y_ref = _A(z) @ x
    y = O.slab_apply_emulated(float(z["C"]), float(z["eta"]), complex(z["omega"]),
                              float(z["h"]), n, cm, x, bounds)
    assert np.linalg.norm(y - y_ref) / np.linalg.norm(y_ref) < 1e-15


def test_shifted_laplace_preconditioner_is_linear():
    n = 24
    om, h, eta = O.problem_params(n, 6, 3.0, 2.0)
    M, Ab = O.shifted_laplace_jacobi(6, 61.0, eta, om, h, n, O.init_c1_mat(.5, .5, n), beta=0.5,
                                      sweeps=3, damping=0.7)
    a, b = rand_complex(n * n, 1), rand_complex(n * n, 2)
    lhs = M @ (2.0 * a - 3j * b)
    rhs = 2.0 * (M @ a) - 3j * (M @ b)
    assert np.linalg.norm(lhs - rhs) / np.linalg.norm(rhs) < 1e-13


def test_marmousi_like_medium_is_deterministic_and_scaled():
    c = media.marmousi_like_c_mat(130)
    assert c.shape == (132, 132)
    assert c.min() >= 0.5 and c.max() <= 1.5 + 1e-12 and c.max() - c.min() > 0.6
    np.testing.assert_array_equal(c, media.marmousi_like_c_mat(130))
    # column-block generation (one row slab's columns) is identical to the full field
    part = media.marmousi_like_c_mat(130, cols=(40, 77), chunk=16)
    np.testing.assert_array_equal(part[:, 40:77], c[:, 40:77])
    assert not part[:, :40].any() and not part[:, 77:].any()
    # velocity increases with depth on average (depth grows toward small y = small row)
    assert c[:20].mean() > c[-20:].mean()


# ------------------------------------------------ the matrix-free C oracle (configs 4 and 5)
def _so():
    from oracle import stencil_oracle as SO
    return SO


@pytest.mark.parametrize("name", ["spmv_n128_const.npz", "spmv_n257_c1.npz"])
def test_c_oracle_spmv_matches_reference(name):
    """oracle/stencil_oracle.c (build_A_matrix's rows without the matrix) against the
    reference's own SpMV outputs."""
    z = load_golden(name)
    n = int(z["n"])
    A = _so().MatrixFreeOperator(int(z["b"]), float(z["C"]), float(z["eta"]),
                                 complex(z["omega"]), float(z["h"]), n, medium(str(z["medium"]), n))
    y = A @ rand_complex(n * n, 0)
    assert np.linalg.norm(y - z["y"]) / np.linalg.norm(z["y"]) < 1e-14


@pytest.mark.parametrize("n,kind", [(1, "const"), (2, "c1"), (33, "c2"), (64, "c1"), (150, "marm"),
                                    (301, "const")])
def test_c_oracle_equals_csr_oracle(n, kind):
    """Row for row the CSR of oracle.build_A_matrix (pinned above by the golden CSRs): apply,
    diagonal and a constant medium given as a scalar, to rounding; and scipy gmres on either
    operator gives the same history (the C oracle stands in for the CSR at 8192^2 and 16384^2)."""
    SO = _so()
    b = min(12, max(1, n // 3))
    om, h, eta = O.problem_params(n, b, 5.0, 2.0)
    cm = media.marmousi_like_c_mat(n) if kind == "marm" else medium(kind, n)
    R = O.build_A_matrix(b, 81.0, eta, om, h, n, cm)
    for A in (SO.MatrixFreeOperator(b, 81.0, eta, om, h, n, cm),) + (
            (SO.MatrixFreeOperator(b, 81.0, eta, om, h, n, 1.0),) if kind == "const" else ()):
        x = rand_complex(n * n, 4)
        y, yr = A @ x, R @ x
        assert np.max(np.abs(y - yr)) <= 1e-15 * np.max(np.abs(yr)) * 4
        d, dr = A.diagonal(), R.diagonal()
        assert np.max(np.abs(d - dr)) <= 1e-15 * np.max(np.abs(dr)) * 4
        assert (A @ x.reshape(-1, 1)).shape == (n * n, 1)
    if n >= 33:
        f = O.init_f1_mat(.5, .125, om, n).ravel()
        _, i1, h1, _ = O.gmres_reference(R, f, M=O.jacobi_preconditioner(R), maxiter=6)
        _, i2, h2, _ = O.gmres_reference(A, f, M=SO.jacobi_preconditioner(A), maxiter=6)
        assert i1 == i2 and np.max(np.abs(h1 - h2) / h1) < 1e-12


def test_c_oracle_shifted_mass_scale():
    """mass_scale 1 + i beta is build_A_matrix(c_mat / sqrt(1 + i beta)) (golden shifted CSR)."""
    z = load_golden("shift_n64.npz")
    n = int(z["n"])
    A = _so().MatrixFreeOperator(int(z["b"]), float(z["C"]), float(z["eta"]),
                                 complex(z["omega"]), float(z["h"]), n, O.init_c1_mat(.5, .5, n),
                                 mass_scale=1 + 1j * float(z["beta"]))
    import scipy.sparse
    R = scipy.sparse.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=(n * n, n * n))
    x = rand_complex(n * n, 6)
    assert np.linalg.norm(A @ x - R @ x) / np.linalg.norm(R @ x) < 1e-14


@pytest.mark.parametrize("K", [5, 7, 20])
def test_gmres_restart_k_is_restart_20(K):
    """scipy gmres (code.py:516, restart 20) stopped by legacy maxiter = K <= 20 inside its first
    cycle is bitwise the restart = K run: the configs-4/5 oracle uses restart K to avoid scipy's
    (restart + 1) x N basis allocation at 16384^2."""
    n = 96
    om, h, eta = O.problem_params(n, 12, 6.0, 2.0)
    A = O.build_A_matrix(12, 81.0, eta, om, h, n, O.init_c1_mat(.5, .5, n))
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    M = O.jacobi_preconditioner(A)
    a = O.gmres_reference(A, f, M=M, rtol=1e-3, restart=20, maxiter=K)
    b = O.gmres_reference(A, f, M=M, rtol=1e-3, restart=K, maxiter=K)
    assert a[1] == b[1] and np.array_equal(a[0], b[0]) and np.array_equal(a[2], b[2])
