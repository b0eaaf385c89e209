"""CPU tier: the C-ABI library loads and exports every symbol the header declares.

No compute calls are made here (there is no GPU in the build container); the one
device call checks that a missing GPU is reported loudly, never silently bypassed.
"""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "helmholtz_amd.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hh_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    for must in ("hh_op_create", "hh_op_apply", "hh_gmres", "hh_ctx_create", "hh_comm_unique_id"):
        assert must in syms


def test_library_exports_every_declared_symbol():
    from helmholtz_preconditioner_amd import _ffi
    lib = ctypes.CDLL(_ffi.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    bound = {name for name, _, _ in _ffi.SIGNATURES}
    assert set(declared_symbols()) <= bound, set(declared_symbols()) - bound
    assert lib.hh_abi_version() == _ffi.ABI_VERSION == 2


def test_library_is_gfx950_code():
    so = os.path.join(ROOT, "helmholtz_preconditioner_amd", "libhelmholtz_amd.so")
    blob = open(so, "rb").read()
    assert b"gfx950" in blob


def test_no_gpu_fails_loudly():
    from helmholtz_preconditioner_amd import _ffi
    n = ctypes.c_int(-1)
    rc = _ffi.lib.hh_device_count(ctypes.byref(n))
    if rc == 0 and n.value > 0:
        pytest.skip("a GPU is visible; loud-failure path not reachable")
    import helmholtz_preconditioner_amd as H
    H.set_default_context(None)
    with pytest.raises(H.HHError):
        H.build_A_matrix(6, 61.0, 6 / 17, 2 * 3.14159 * 2 + 2j, 1 / 17, 16, H.constant_c_mat(16))


def test_error_message_roundtrip():
    from helmholtz_preconditioner_amd import _ffi
    rc = _ffi.lib.hh_ctx_create(0, 3, 2, None, 1, ctypes.byref(ctypes.c_void_p()))
    assert rc == -1  # HH_ERR_INVALID: rank >= world
    assert b"rank" in _ffi.lib.hh_last_error()


_KNOB_CHILD = ("import sys, json; sys.path.insert(0, sys.argv[1]); "
               "import helmholtz_preconditioner_amd as H; print(json.dumps(H.knobs()))")


@pytest.mark.parametrize("env,want", [({}, {}),
                                      ({"HH_LAG_RED": "0", "HH_SLK": "3"},
                                       {"HH_LAG_RED": 0, "HH_SLK": 3}),
                                      ({"HH_CYCLE_MERGE": "1"}, {})])
def test_knobs_read_once_and_reported(env, want):
    """Every HH_* knob is read once into one struct (knobs.cpp) and reported by hh_knobs_json:
    only those off the shipped path (bench.py prints them into its line's config), so a default
    run reports {} and a knob set to its default is not reported either."""
    import json
    import subprocess
    import sys
    clean = {k: v for k, v in os.environ.items() if not k.startswith("HH_")}
    r = subprocess.run([sys.executable, "-c", _KNOB_CHILD, ROOT], env=dict(clean, **env),
                       capture_output=True, text=True, timeout=120, check=True)
    got = json.loads(r.stdout.strip().splitlines()[-1])
    assert {k: v["value"] for k, v in got.items()} == want


@pytest.mark.parametrize("env,msg", [({"HH_FUSED_KEEP": "4"}, "HH_FUSED_KEEP=4"),
                                     ({"HH_SLK": "two"}, "HH_SLK=two: not an integer")])
def test_malformed_knob_fails_loudly(env, msg):
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "-c", _KNOB_CHILD, ROOT], env=dict(os.environ, **env),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and msg in r.stderr, r.stderr[-2000:]
