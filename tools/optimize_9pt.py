"""Dispersion-optimal weights of the 9-point operator.

The scheme (csrc/stencil.hip, oracle.build_A9_matrix) is
    alpha * (5-point Laplacian) + (1 - alpha) * (line-averaged second differences)
    + (w h / c)^2 (c u_C + d sum(edges) + e sum(corners)),   e = (1 - c - 4d) / 4,
the family of Chen, Cheng, Feng & Wu's optimal 9-point PML scheme (2013).  This fits
(alpha, c, d) by least squares on the normalised phase velocity of the constant-medium
scheme over 4 ... 400 points per wavelength and propagation angles 0 ... 45 degrees, and
prints the worst-case phase error against the 5-point scheme's.  CPU only.
usage: python tools/optimize_9pt.py
"""
import os
import sys

import numpy as np
from scipy.optimize import least_squares

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle.helmholtz_oracle import STENCIL9_WEIGHTS, phase_velocity_9pt  # noqa: E402


def main():
    inv_g = np.linspace(0.0025, 0.25, 100)
    phi = np.linspace(0, np.pi / 4, 16)
    IG, PH = np.meshgrid(inv_g, phi)
    res = lambda p: (phase_velocity_9pt(p, 1 / IG, PH) - 1).ravel()  # noqa: E731
    fit = least_squares(res, [0.5, 0.6, 0.1], xtol=1e-14, ftol=1e-14)
    a, c, d = fit.x
    print(f"least-squares fit: alpha={a:.7f} c={c:.7f} d={d:.7f} e={(1 - c - 4 * d) / 4:.7f}")
    print(f"shipped defaults : alpha={STENCIL9_WEIGHTS[0]} c={STENCIL9_WEIGHTS[1]} "
          f"d={STENCIL9_WEIGHTS[2]}")
    print("points/wavelength  max|v/c - 1| 5-point   9-point (shipped)")
    for G in (4, 5, 6, 8, 10, 20, 40):
        e5 = np.abs(phase_velocity_9pt((1, 1, 0), G, phi) - 1).max()
        e9 = np.abs(phase_velocity_9pt(STENCIL9_WEIGHTS, G, phi) - 1).max()
        print(f"{G:17d}  {e5:20.2e}  {e9:10.2e}")


if __name__ == "__main__":
    main()
