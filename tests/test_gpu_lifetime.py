"""GPU tier: handle lifetimes of the C ABI (context > operator > vector).

Releasing a handle never frees an object that another live object still uses: a context
outlives its operators and an operator its vectors, whatever order the caller (or a
garbage collector) releases them in -- and no stale HIP error leaks into a later call.
"""
import numpy as np
import pytest

import helmholtz_preconditioner_amd as H
from conftest import rand_complex

pytestmark = pytest.mark.gpu


def _op(ctx, n=40):
    om, h, eta = H.problem_params(n, 6, 3.0, 2.0)
    return H.build_A_matrix(6, 81.0, eta, om, h, n, H.init_c1_mat(.5, .5, n), context=ctx)


def test_release_context_before_operator_and_vectors():
    ctx = H.Context(device=0)
    A = _op(ctx)
    x = A.vector(rand_complex(A.local_size, 0))
    y = A.vector()
    ref = A @ x.download()
    ctx.close()                 # the operator keeps the context alive
    A.apply_device(x, y)
    np.testing.assert_array_equal(y.download(), ref)
    A.close()                   # the vectors keep the operator alive
    y.upload(np.zeros(A.local_size, dtype=np.complex128))
    assert not np.any(y.download())
    x.close()
    y.close()                   # last reference: operator and context freed here


def test_no_stale_error_after_out_of_order_teardown():
    for _ in range(3):
        ctx = H.Context(device=0)
        A = _op(ctx)
        v = A.vector()
        del ctx
        A.close()
        del v
    # a fresh operator on a fresh context works and reports no leftover error
    c2 = H.Context(device=0)
    B = _op(c2, 33)
    xb = rand_complex(B.local_size, 1)
    assert np.all(np.isfinite(B @ xb))
