"""Bitwise A/B of the device GMRES between two builds of the library (HH_LIB_PATH):
`ab_gmres_bits.py dump OUT.npz` records histories and fields of a fixed set of solves;
`ab_gmres_bits.py compare A.npz B.npz` reports whether every array is bit-identical."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(path):
    import helmholtz_preconditioner_amd as H
    out = {}
    for n, kind, reorth, maxiter in [(128, "none", False, 60), (300, "jacobi", False, 47),
                                     (300, "jacobi", True, 30), (257, "sl", False, 45),
                                     (1024, "jacobi", False, 40)]:
        om, h, eta = H.problem_params(n, 12, 8.0, 2.0)
        A = H.build_A_matrix(12, 81.0, eta, om, h, n, H.init_c1_mat(.5, .5, n))
        f = H.init_f1_mat(.5, .125, om, n).ravel()
        M = {"none": None, "jacobi": "jacobi",
             "sl": H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7)}[kind]
        hist = []
        x, info = H.gmres(A, f, rtol=1e-14, restart=20, maxiter=maxiter, M=M, reorth=reorth,
                          callback=hist.append, callback_type="legacy")
        key = f"n{n}_{kind}_{int(reorth)}"
        out[key + "_hist"] = np.array(hist)
        out[key + "_x"] = x
        out[key + "_info"] = np.array(info)
    np.savez(path, **out)


def compare(a, b):
    za, zb = np.load(a), np.load(b)
    bad = [k for k in za.files if not np.array_equal(za[k], zb[k])]
    print("bit-identical" if not bad else f"DIFFER: {bad}", f"({len(za.files)} arrays)")
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
