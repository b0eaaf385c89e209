"""Test configuration.

Tiers:
  * CPU (`-m "not gpu"`): the oracle against the golden vectors generated from the
    reference itself, host logic, the row-slab decomposition over gloo, and that the
    C-ABI library loads and exports every symbol include/helmholtz_amd.h declares.
  * GPU (`-m gpu`): parity of the HIP path (through the C ABI) against the oracle and
    the golden vectors.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def rand_complex(n_total, seed=0):
    rng = np.random.default_rng(seed)
    return rng.standard_normal(n_total) + 1j * rng.standard_normal(n_total)


def medium(kind, n):
    from oracle import helmholtz_oracle as O
    if kind == "c1":
        return O.init_c1_mat(.5, .5, n)
    if kind == "c2":
        return O.init_c2_mat(n)
    if kind == "const":
        return np.ones((n + 2, n + 2))
    raise ValueError(kind)


@pytest.fixture(scope="session")
def golden():
    return load_golden


def _ensure_native_library():
    """Build libhelmholtz_amd.so if a fresh checkout lacks it (hipcc cross-compiles
    for gfx950 without a GPU); the package refuses to import without it."""
    so = os.path.join(ROOT, "helmholtz_preconditioner_amd", "libhelmholtz_amd.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-s", "-j8", "-C",
                        os.path.join(ROOT, "helmholtz_preconditioner_amd", "csrc")], check=True)


def _ensure_c_oracle():
    """Build the C oracle (oracle/build/libhh_oracle.so, test infrastructure) if missing."""
    so = os.path.join(ROOT, "oracle", "build", "libhh_oracle.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


_ensure_native_library()
_ensure_c_oracle()
