"""CPU tier, SURVEY row F3: velocity loaders, resampling and solution output (host logic).

The reference has no loaders (its media are analytic, code.py:39-66); the contract here
is the reference's c_mat convention (c_mat[r, q] = c(x = q h, y = r h), code.py:41-43) and
its solution view flipud(Re u) (code.py:527-529).
"""
import numpy as np
import pytest

import helmholtz_preconditioner_amd as H
from helmholtz_preconditioner_amd import io as hio


def test_c_mat_roundtrip_npy_npz_raw(tmp_path):
    n = 13
    c = H.init_c1_mat(.5, .5, n)
    H.save_c_mat(tmp_path / "c.npy", c)
    np.testing.assert_array_equal(H.load_c_mat(tmp_path / "c.npy", n), c)
    np.savez(tmp_path / "c.npz", c_mat=c)
    np.testing.assert_array_equal(H.load_c_mat(tmp_path / "c.npz"), c)
    c.astype("<f8").tofile(tmp_path / "c.bin")
    np.testing.assert_array_equal(H.load_c_mat(tmp_path / "c.bin", n, dtype="float64"), c)
    c.astype("<f4").tofile(tmp_path / "c32.bin")
    got = H.load_c_mat(tmp_path / "c32.bin", n, dtype="f4")
    assert got.dtype == np.float64
    np.testing.assert_array_equal(got, c.astype(np.float32).astype(np.float64))


def test_c_mat_rejects_bad_input(tmp_path):
    n = 8
    with pytest.raises(ValueError):
        H.load_c_mat(tmp_path / "missing.bin", n)          # raw without dtype
    np.save(tmp_path / "wrong.npy", np.ones((n + 1, n + 2)))
    with pytest.raises(ValueError):
        H.load_c_mat(tmp_path / "wrong.npy", n)
    bad = np.ones((n + 2, n + 2))
    bad[3, 3] = -1.0
    np.save(tmp_path / "neg.npy", bad)
    with pytest.raises(ValueError):
        H.load_c_mat(tmp_path / "neg.npy", n)
    np.ones(5).tofile(tmp_path / "short.bin")
    with pytest.raises(ValueError):
        H.load_c_mat(tmp_path / "short.bin", n, dtype="f8")
    # pickled object arrays are refused, never unpickled
    np.save(tmp_path / "obj.npy", np.array([{"a": 1}], dtype=object), allow_pickle=True)
    with pytest.raises(ValueError):
        H.load_c_mat(tmp_path / "obj.npy")


def test_resample_orientation_and_exactness():
    # a model that is linear in depth and x is reproduced exactly by bilinear resampling
    nz, nx, n = 41, 57, 30
    depth = np.linspace(0, 1, nz)[:, None]
    x = np.linspace(0, 1, nx)[None, :]
    model = 1.0 + 2.0 * depth + 0.5 * x
    c = H.resample_velocity(model, n)
    t = np.linspace(0, 1, n + 2)
    expect = 1.0 + 2.0 * (1.0 - t)[:, None] + 0.5 * t[None, :]   # row r: y = r h, depth = 1 - y
    np.testing.assert_allclose(c, expect, rtol=0, atol=1e-13)
    # surface (model row 0) lands on the Dirichlet side y = 1 (last c_mat row)
    assert c[-1, 0] == pytest.approx(model[0, 0]) and c[0, 0] == pytest.approx(model[-1, 0])
    # affine range mapping
    s = H.resample_velocity(model, n, vmin=0.5, vmax=1.5)
    assert s.min() == pytest.approx(0.5) and s.max() == pytest.approx(1.5)
    with pytest.raises(ValueError):
        H.resample_velocity(model, n, vmin=0.5)


def test_resample_constant_and_marmousi_like_grid(tmp_path):
    n = 20
    np.testing.assert_array_equal(H.resample_velocity(np.full((7, 9), 2.5), n), np.full((n + 2, n + 2), 2.5))
    # a model on exactly the c_mat nodes (depth-major) resamples to itself
    m = H.marmousi_like_c_mat(n)
    model = m[::-1]              # [depth][x]: row 0 = y = 1 surface
    np.save(tmp_path / "model.npy", model)
    np.testing.assert_allclose(H.load_velocity_model(tmp_path / "model.npy", n), m, rtol=0, atol=1e-14)


def test_solution_roundtrip_and_image(tmp_path):
    n = 9
    rng = np.random.default_rng(0)
    u = rng.standard_normal(n * n) + 1j * rng.standard_normal(n * n)
    H.save_solution(tmp_path / "u.npz", u, n, wave_num=4.0, omega=2 * np.pi * 4 + 2j, info=0)
    u2, n2, params = H.load_solution(tmp_path / "u.npz")
    np.testing.assert_array_equal(u2, u)
    assert n2 == n and params["wave_num"] == 4.0 and params["info"] == 0
    assert params["omega"] == 2 * np.pi * 4 + 2j
    img = H.solution_image(u, n)
    np.testing.assert_array_equal(img, np.flipud(np.real(u.reshape(n, n))))
    with pytest.raises(ValueError):
        H.save_solution(tmp_path / "bad.npz", u[:-1], n)


def test_plot_solution_writes_png(tmp_path):
    pytest.importorskip("matplotlib")
    n = 8
    u = np.arange(n * n) * (1 + 1j)
    out = tmp_path / "u.png"
    hio.plot_solution(u, n, 4.0, 81.0, path=out)
    assert out.exists() and out.stat().st_size > 1000
