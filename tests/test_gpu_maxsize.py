"""GPU tier: the largest single-GPU configuration (BASELINE config 5, n = 16384, 268M unknowns,
4.3 GB per vector) for both stencils, checked point-wise against the oracle's formulas
(oracle.apply_at_points: no assembly, which would need 27 GB of CSR) at the grid's corners,
edges, the PML / interior boundary rows and a random sample.  Tolerance as the other apply
tests: 1e-12 relative to the row-sample norm.
"""
import numpy as np
import pytest

import helmholtz_preconditioner_amd as H
from oracle import helmholtz_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = H.Context(device=0)
    H.set_default_context(c)
    yield c
    H.set_default_context(None)


def _sample(n, b):
    rng = np.random.default_rng(16384)
    rows = [0, 1, b - 1, b, b + 1, n // 2, n - b - 1, n - b, n - 2, n - 1]
    cols = [0, 1, b - 1, b, b + 1, n // 2, n - b - 1, n - b, n - 2, n - 1]
    P = [j * n + i for j in rows for i in cols]
    P += list(rng.integers(0, n * n, 2000))
    return np.unique(np.array(P, dtype=np.int64))


@pytest.mark.parametrize("stencil", [5, 9])
def test_config5_apply_pointwise(ctx, stencil):
    n, b = 16384, 12
    om, h, eta = O.problem_params(n, b, 800.0, 2.0)
    A = H.build_A_matrix(b, 81.0, eta, om, h, n, H.constant_c_mat(n),
                         context=ctx, stencil=stencil)
    assert A.constant_medium and A.local_size == n * n
    x, y = A.vector(), A.vector()
    x.fill_hash(99)
    A.apply_device(x, y)
    xh, yh = x.download(), y.download()
    del x, y
    P = _sample(n, b)
    ref = O.apply_at_points(81.0, eta, om, h, n, lambda I, J: np.ones(np.shape(I)), xh, P,
                            stencil=stencil)
    err = np.linalg.norm(yh[P] - ref) / np.linalg.norm(ref)
    assert err < 1e-12, err
    A.close()
