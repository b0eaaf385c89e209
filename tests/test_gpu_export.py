"""GPU tier, SURVEY row F2: the CSR export (``DeviceOperator.to_csr``, hh_op_export_csr).

The exported matrix must be the reference's ``build_A_matrix`` (code.py:202-219):
identical structure (indptr, indices: exact) and values within 1e-13 relative per entry
(golden CSR written by the reference itself, tests/golden/coef_*.npz).  It must also be
exactly the operator the stencil applies: the kernel evaluates the coefficients with the
stencil's own operation order, so a slab decomposition exports bit-identical rows.
"""
import numpy as np
import pytest
import scipy.sparse

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


def _params(z):
    return int(z["b"]), float(z["C"]), float(z["eta"]), complex(z["omega"]), float(z["h"]), int(z["n"])


@pytest.mark.parametrize("name", ["coef_n16_c1.npz", "coef_n33_c2.npz", "coef_n64_const.npz",
                                  "coef_n64_c1.npz"])
def test_to_csr_matches_reference_golden(ctx, name):
    z = load_golden(name)
    b, C, eta, om, h, n = _params(z)
    A = H.build_A_matrix(b, C, eta, om, h, n, medium(str(z["medium"]), n), context=ctx)
    M = A.to_csr()
    assert isinstance(M, scipy.sparse.csr_matrix)
    assert M.shape == (n * n, n * n) and M.nnz == 5 * n * n - 4 * n == len(z["data"])
    assert M.indices.dtype == np.int32
    np.testing.assert_array_equal(M.indptr, z["indptr"])
    np.testing.assert_array_equal(M.indices, z["indices"])
    rel = np.abs(M.data - z["data"]) / np.abs(z["data"])
    assert rel.max() < 1e-13, rel.max()
    # the exported matrix is the applied operator
    x = rand_complex(n * n, 3)
    y = A @ x
    assert np.linalg.norm(M @ x - y) / np.linalg.norm(y) < 1e-14


@pytest.mark.parametrize("n,kind", [(1, "const"), (2, "c1"), (5, "c1"), (300, "c1"), (1024, "const")])
def test_to_csr_structure_and_values_vs_oracle(ctx, n, kind):
    b = min(12, max(1, n // 4))
    om, h, eta = H.problem_params(n, b, 4.0, 2.0)
    cm = medium(kind, n)
    A = H.build_A_matrix(b, 81.0, eta, om, h, n, cm, context=ctx)
    M = A.to_csr()
    R = O.build_A_matrix(b, 81.0, eta, om, h, n, cm).tocsr()
    R.sort_indices()
    assert M.nnz == R.nnz == 5 * n * n - 4 * n
    np.testing.assert_array_equal(M.indptr, R.indptr)
    np.testing.assert_array_equal(M.indices, R.indices)
    assert (np.abs(M.data - R.data) / np.abs(R.data)).max() < 1e-13


def test_to_csr_int64_indices_and_slabs_bit_identical(ctx):
    n = 97
    om, h, eta = H.problem_params(n, 12, 6.0, 2.0)
    cm = O.init_c2_mat(n)
    A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm, context=ctx)
    M32 = A.to_csr()
    M64, ms = A.to_csr(index_dtype=np.int64, return_kernel_ms=True)
    assert ms >= 0.0
    assert M64.indices.dtype == np.int64 and M64.indptr.dtype == np.int64
    np.testing.assert_array_equal(M64.indices, M32.indices)
    np.testing.assert_array_equal(M64.data, M32.data)
    # three virtual slabs on one device: the same rows, bit for bit
    c3 = H.Context(device=0, virtual_slabs=3)
    A3 = H.build_A_matrix(12, 81.0, eta, om, h, n, cm, context=c3)
    M3 = A3.to_csr()
    np.testing.assert_array_equal(M3.indptr, M32.indptr)
    np.testing.assert_array_equal(M3.indices, M32.indices)
    np.testing.assert_array_equal(M3.data, M32.data)
    A3.close()
    c3.close()


def test_to_csr_shifted_operator_matches_golden(ctx):
    """build_A_matrix(..., c_mat / sqrt(1 + 0.5i)) -- the shifted-Laplace operator."""
    z = load_golden("shift_n64.npz")
    b, C, eta, om, h, n = _params(z)
    cm = medium(str(z["medium"]), n) / np.sqrt(1 + float(z["beta"]) * 1j)
    A = H.build_A_matrix(b, C, eta, om, h, n, cm, context=ctx)
    M = A.to_csr()
    np.testing.assert_array_equal(M.indptr, z["indptr"])
    np.testing.assert_array_equal(M.indices, z["indices"])
    assert (np.abs(M.data - z["data"]) / np.abs(z["data"])).max() < 1e-12
