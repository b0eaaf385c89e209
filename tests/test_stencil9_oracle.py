"""CPU tier: the 9-point operator's restatement.

The reference has no 9-point operator (code.py:216-218 assembles 5 points), so nothing
from the reference pins this one: "parity unpinned" by the reference.  The oracle is
instead pinned by properties that any correct implementation of the scheme must have:
  * weights (1, 1, 0) reproduce the reference's 5-point build_A_matrix (itself pinned by
    the golden CSR generated from code.py),
  * structure (canonical CSR, nnz = (3n-2)^2),
  * second-order consistency (observed order of the truncation error ~2, PML off),
  * the mass weights sum to 1 (row sums of the PML-free operator on constants),
  * dispersion: the shipped weights give <= 0.42 % phase error at >= 4 points per
    wavelength (5-point: 10 %), and the oracle's operator has that symbol.
"""
import numpy as np
import pytest
import scipy.sparse

from conftest import load_golden, medium, rand_complex
from oracle import helmholtz_oracle as O

W9 = O.STENCIL9_WEIGHTS


def _params(z):
    return int(z["b"]), float(z["C"]), float(z["eta"]), complex(z["omega"]), float(z["h"]), int(z["n"])


@pytest.mark.parametrize("name", ["coef_n16_c1.npz", "coef_n33_c2.npz", "coef_n64_const.npz"])
def test_unit_weights_reduce_to_reference_5pt(name):
    z = load_golden(name)
    b, C, eta, om, h, n = _params(z)
    Aref = scipy.sparse.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=(n * n, n * n))
    A9 = O.build_A9_matrix(b, C, eta, om, h, n, medium(str(z["medium"]), n), weights=(1.0, 1.0, 0.0))
    D = (A9 - Aref).tocoo()
    assert np.max(np.abs(D.data), initial=0) <= 1e-15 * np.max(np.abs(Aref.data))


@pytest.mark.parametrize("n", [1, 2, 3, 17])
def test_structure(n):
    om, h, eta = O.problem_params(n, 1, 3.0, 2.0)
    A = O.build_A9_matrix(1, 81.0, eta, om, h, n, medium("c1", n))
    assert A.nnz == (3 * n - 2) ** 2
    assert A.has_sorted_indices
    # row p couples exactly to the in-grid points of its 3x3 neighbourhood
    p = (n // 2) * n + n // 2
    cols = A.indices[A.indptr[p]:A.indptr[p + 1]]
    i, j = p % n, p // n
    want = sorted((j + dj) * n + i + di for dj in (-1, 0, 1) for di in (-1, 0, 1)
                  if 0 <= i + di < n and 0 <= j + dj < n)
    assert list(cols) == want


def _truncation_error(n, weights):
    """max |A9 u - (Lap u + (w/c)^2 u)| at the interior for a smooth u, PML off (C = 0)."""
    om = 7.0 + 0.0j
    h = 1.0 / (n + 1)
    cm = np.ones((n + 2, n + 2)) * 1.3
    A = O.build_A9_matrix(1, 0.0, h, om, h, n, cm, weights=weights)
    x = np.arange(1, n + 1) * h
    X, Y = np.meshgrid(x, x)                        # [j, i]: X = x1 = i h, Y = x2 = j h
    u = np.sin(np.pi * X) * np.sin(2 * np.pi * Y)   # zero on the boundary
    exact = (-(np.pi ** 2) - (2 * np.pi) ** 2 + (om / 1.3) ** 2) * u
    return np.max(np.abs((A @ u.ravel()).reshape(n, n) - exact))


@pytest.mark.parametrize("weights", [W9, (1.0, 1.0, 0.0), (0.5, 0.7, 0.05)])
def test_second_order_consistency(weights):
    e1, e2 = _truncation_error(31, weights), _truncation_error(63, weights)
    order = np.log2(e1 / e2)
    assert 1.8 < order < 2.3, order


def test_mass_weights_sum_to_one():
    n = 20
    om = 5.0 + 0.0j
    h = 1.0 / (n + 1)
    A = O.build_A9_matrix(1, 0.0, h, om, h, n, np.full((n + 2, n + 2), 2.0))
    rs = (A @ np.ones(n * n)).reshape(n, n)[1:-1, 1:-1]   # interior: Laplacian of 1 is 0
    np.testing.assert_allclose(rs, (om / 2.0) ** 2, rtol=1e-11)


def test_dispersion_of_shipped_weights():
    phi = np.linspace(0, np.pi / 4, 31)
    for G in (4, 5, 6, 8, 10, 20, 40):
        e9 = np.abs(O.phase_velocity_9pt(W9, G, phi) - 1).max()
        e5 = np.abs(O.phase_velocity_9pt((1, 1, 0), G, phi) - 1).max()
        assert e9 < 4.2e-3 and e9 < e5 / 8, (G, e9, e5)


def test_operator_symbol_matches_dispersion_formula():
    """A9 (PML off, constant c) applied to a plane wave e^{i k.x} at an interior point equals
    the symbol phase_velocity_9pt is derived from."""
    n = 40
    h = 1.0 / (n + 1)
    om = 11.0 + 0.0j
    A = O.build_A9_matrix(1, 0.0, h, om, h, n, np.ones((n + 2, n + 2)))
    kh, phi = 2 * np.pi / 6, 0.3
    t, s = kh * np.cos(phi), kh * np.sin(phi)
    I, J = np.meshgrid(np.arange(n), np.arange(n))
    u = np.exp(1j * (t * I + s * J))
    p = (n // 2) * n + n // 2
    got = (A @ u.ravel())[p] / u.ravel()[p]
    a, c, d = W9
    e = (1 - c - 4 * d) / 4
    L = a * (2 * np.cos(t) + 2 * np.cos(s) - 4) + (1 - a) * (4 * np.cos(t) * np.cos(s) - 2 * np.cos(t) - 2 * np.cos(s))
    m = c + 2 * d * (np.cos(t) + np.cos(s)) + 4 * e * np.cos(t) * np.cos(s)
    np.testing.assert_allclose(got, L / h ** 2 + om ** 2 * m, rtol=1e-12)


def test_shifted_9pt_operator_is_mass_scaled():
    """c_mat / sqrt(1 + i beta) multiplies exactly the mass part (M terms) by 1 + i beta."""
    n, beta = 24, 0.5
    om, h, eta = O.problem_params(n, 4, 3.0, 2.0)
    cm = medium("c1", n)
    A = O.build_A9_matrix(4, 81.0, eta, om, h, n, cm)
    Ab = O.build_A9_matrix(4, 81.0, eta, om, h, n, cm / np.sqrt(1 + 1j * beta))
    Z = O.build_A9_matrix(4, 81.0, eta, om, h, n, cm * 1e30)     # mass-free part
    x = rand_complex(n * n, 3)
    np.testing.assert_allclose(Ab @ x, Z @ x + (1 + 1j * beta) * ((A - Z) @ x), rtol=1e-11,
                               atol=1e-9 * np.abs(A @ x).max())
