"""On-disk inputs and outputs around the hot path.

Reference: the velocity and forcing initialisers (code.py:39-66, 388-408) produce an
(n+2) x (n+2) float64 ``c_mat`` in the meshgrid convention c_mat[r, q] = c(x = q h,
y = r h), and the result is shown as ``np.flipud(np.real(u.reshape(n, n)))`` with
``extent=[0, 1, 0, 1]`` (code.py:527-539).  This module lets a real velocity model (for
example a local copy of Marmousi) replace the synthetic ones and writes the solution:

* :func:`load_c_mat` -- a velocity file already in the reference's (n+2)^2 c_mat
  convention (``.npy``, or raw little-endian float32/float64 with a given shape);
* :func:`load_velocity_model` / :func:`resample_velocity` -- a geophysical model laid
  out [depth][x] (row 0 = surface, depth increasing downward, like the Marmousi grid),
  resampled bilinearly onto the c_mat nodes.  The surface is y = 1 (the Dirichlet side,
  code.py:20-25: the PML of sigma2 sits at y <= eta), i.e. depth = 1 - y -- the same
  orientation as :func:`helmholtz_preconditioner_amd.marmousi_like_c_mat`;
* :func:`save_solution` / :func:`load_solution` -- the field with its problem parameters
  (``.npz``, no pickles), and :func:`solution_image` / :func:`plot_solution` -- the
  reference's flipud(Re u) view.

Loaders never execute anything from a file: ``numpy.load(allow_pickle=False)`` and raw
``numpy.fromfile``.
"""
from __future__ import annotations

import os

import numpy as np

_RAW_DTYPES = {"f4": np.dtype("<f4"), "float32": np.dtype("<f4"),
               "f8": np.dtype("<f8"), "float64": np.dtype("<f8")}


def _read_array(path, shape=None, dtype=None):
    ext = os.path.splitext(str(path))[1].lower()
    if ext == ".npy":
        a = np.load(path, allow_pickle=False)
        if shape is not None and tuple(a.shape) != tuple(shape):
            raise ValueError(f"{path}: shape {a.shape}, expected {tuple(shape)}")
        return np.asarray(a)
    if ext == ".npz":
        z = np.load(path, allow_pickle=False)
        keys = list(z.files)
        key = "c_mat" if "c_mat" in keys else ("velocity" if "velocity" in keys else None)
        if key is None:
            if len(keys) != 1:
                raise ValueError(f"{path}: expected one array or a 'c_mat'/'velocity' entry, got {keys}")
            key = keys[0]
        return np.asarray(z[key])
    # raw binary: needs an explicit shape and element type
    if shape is None or dtype is None:
        raise ValueError(f"{path}: raw files need shape=(rows, cols) and dtype='float32'|'float64'")
    dt = _RAW_DTYPES.get(str(dtype), None) if not isinstance(dtype, np.dtype) else dtype.newbyteorder("<")
    if dt is None:
        raise ValueError(f"unsupported raw dtype {dtype!r}")
    count = int(np.prod(shape))
    size = os.path.getsize(path)
    if size != count * dt.itemsize:
        raise ValueError(f"{path}: {size} bytes, expected {count * dt.itemsize} for {shape} {dt}")
    return np.fromfile(path, dtype=dt, count=count).reshape(shape)


def _check_velocity(c, what):
    c = np.asarray(c, dtype=np.float64)
    if not np.all(np.isfinite(c)):
        raise ValueError(f"{what}: non-finite velocity values")
    if np.any(c <= 0):
        raise ValueError(f"{what}: velocities must be positive")
    return c


def load_c_mat(path, n=None, *, shape=None, dtype=None):
    """A velocity file in the reference's c_mat convention ((n+2) x (n+2), c_mat[r, q] =
    c(x = q h, y = r h)), ready for ``build_A_matrix``.  ``n`` (optional) checks the size."""
    if shape is None and n is not None:
        shape = (n + 2, n + 2)
    c = _read_array(path, shape, dtype)
    if c.ndim != 2 or c.shape[0] != c.shape[1]:
        raise ValueError(f"{path}: c_mat must be square, got {c.shape}")
    if n is not None and c.shape != (n + 2, n + 2):
        raise ValueError(f"{path}: c_mat is {c.shape}, expected {(n + 2, n + 2)}")
    return np.ascontiguousarray(_check_velocity(c, str(path)))


def resample_velocity(model, n, *, vmin=None, vmax=None):
    """Bilinear resampling of a [depth][x] model onto the (n+2)^2 c_mat nodes.

    The model spans the unit square: model[0, :] is the surface (y = 1), model[-1, :] the
    deepest row (y = 0); columns run x = 0 .. 1.  Node (r, q) of c_mat sits at x = q h,
    y = r h, depth = 1 - y.  ``vmin``/``vmax`` (both or neither) map the model's range
    affinely onto [vmin, vmax] -- the BASELINE "scaled to [0.5, 1.5]" convention.
    """
    m = _check_velocity(model, "model")
    if m.ndim != 2 or min(m.shape) < 1:
        raise ValueError(f"model must be 2-D, got {m.shape}")
    if (vmin is None) != (vmax is None):
        raise ValueError("give both vmin and vmax, or neither")
    nz, nx = m.shape
    t = np.linspace(0.0, 1.0, n + 2)
    # fractional model coordinates of every node
    zc = (1.0 - t) * (nz - 1)          # row r of c_mat -> depth index
    xc = t * (nx - 1)                  # column q -> x index
    z0 = np.clip(np.floor(zc).astype(np.int64), 0, max(nz - 2, 0))
    x0 = np.clip(np.floor(xc).astype(np.int64), 0, max(nx - 2, 0))
    z1, x1 = np.minimum(z0 + 1, nz - 1), np.minimum(x0 + 1, nx - 1)
    wz = (zc - z0)[:, None]
    wx = (xc - x0)[None, :]
    c = ((1 - wz) * ((1 - wx) * m[z0][:, x0] + wx * m[z0][:, x1])
         + wz * ((1 - wx) * m[z1][:, x0] + wx * m[z1][:, x1]))
    if vmin is not None:
        lo, hi = float(m.min()), float(m.max())
        c = np.full_like(c, 0.5 * (vmin + vmax)) if hi == lo else vmin + (vmax - vmin) * (c - lo) / (hi - lo)
    return np.ascontiguousarray(c)


def load_velocity_model(path, n, *, shape=None, dtype=None, vmin=None, vmax=None):
    """Read a [depth][x] velocity model (``.npy``/``.npz``/raw) and resample it to the
    (n+2)^2 c_mat of an n x n interior grid (see :func:`resample_velocity`)."""
    return resample_velocity(_read_array(path, shape, dtype), n, vmin=vmin, vmax=vmax)


def save_c_mat(path, c_mat):
    """Write a c_mat as ``.npy`` (the format :func:`load_c_mat` reads back)."""
    np.save(path, np.ascontiguousarray(_check_velocity(c_mat, "c_mat")), allow_pickle=False)


def solution_image(u, n):
    """The reference's display of a solution: ``np.flipud(np.real(u.reshape(n, n)))``
    (code.py:527-529), row 0 at the top of the picture (y = 1)."""
    return np.flipud(np.real(np.asarray(u).reshape(n, n)))


def save_solution(path, u, n, **params):
    """Write the field u (length n^2, the reference's p = (j-1) n + (i-1) order) and its
    problem parameters (scalars / small arrays) to an ``.npz``."""
    u = np.asarray(u, dtype=np.complex128).ravel()
    if u.size != n * n:
        raise ValueError(f"u has {u.size} values, expected {n * n}")
    clean = {}
    for k, v in params.items():
        a = np.asarray(v)
        if a.dtype == object:
            raise TypeError(f"parameter {k!r} is not a plain number/array")
        clean[k] = a
    np.savez(path, u=u, n=np.int64(n), **clean)


def load_solution(path):
    """(u, n, params) from :func:`save_solution`."""
    z = np.load(path, allow_pickle=False)
    params = {k: (z[k].item() if z[k].ndim == 0 else z[k]) for k in z.files if k not in ("u", "n")}
    return z["u"], int(z["n"]), params


def plot_solution(u, n, wave_num, const, path=None, title_extra=""):
    """The reference's solution figure (code.py:527-539): imshow of flipud(Re u) on
    [0, 1]^2 with the same title, saved to ``path`` (or shown).  Needs matplotlib."""
    import matplotlib
    if path is not None:
        matplotlib.use("Agg", force=False)
    import matplotlib.pyplot as plt
    fig = plt.figure()
    plt.imshow(solution_image(u, n), extent=[0, 1, 0, 1])
    plt.xlabel("x")
    plt.ylabel("y")
    plt.title(f"N = {n}$^2$ \n $\\omega /(2\\pi)$ = {wave_num} \n const = {const} \n Real(u)"
              + title_extra)
    plt.colorbar()
    plt.tight_layout()
    if path is not None:
        fig.savefig(path)
        plt.close(fig)
    else:  # pragma: no cover - interactive
        plt.show()
    return fig
