"""Bitwise A/B of two builds of libhelmholtz_amd.so on GMRES solves (histories, fields, it/s).
usage: python tools/ab_lib_bits.py OTHER_LIB_PATH OUT_DIR
Runs the case list in a child process per library (HH_LIB_PATH), then compares."""
import hashlib
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [  # (name, n, medium, precond, krylov mode, stencil, maxiter)
    ("c2_jacobi_1024", 1024, "const", "jacobi", "auto", 5, 45),
    ("c3_sl_4096", 4096, "marmousi", "sl", "auto", 5, 25),
    ("lag_sl_700", 700, "marmousi", "sl", "one", 5, 45),
    ("lag_none_600", 600, "const", None, "one", 5, 45),
    ("s9_sl_1100", 1100, "marmousi", "sl", "auto", 9, 30),
    ("none_300_r7", 300, "const", None, "auto", 5, 40),
]


def child(out_dir, tag):
    sys.path.insert(0, ROOT)
    import helmholtz_preconditioner_amd as H
    res = {}
    for name, n, med, pre, mode, st, K in CASES:
        om, h, eta = H.problem_params(n, 12, max(3.0, n / 40.0), 2.0)
        cm = H.marmousi_like_c_mat(n) if med == "marmousi" else H.constant_c_mat(n)
        A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm, stencil=st)
        A.krylov_mode(mode)
        M = H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7) if pre == "sl" else pre
        f = H.init_f1_mat(.5, .125, om, n).ravel()
        restart = 7 if name.endswith("r7") else 20
        x, info, hist = H.gmres(A, f, rtol=1e-12, restart=restart, maxiter=K, M=M,
                                callback=lambda r: None, callback_type="legacy",
                                return_history=True)
        t0 = time.perf_counter()
        H.gmres(A, f, rtol=1e-12, restart=restart, maxiter=K, M=M, callback=lambda r: None,
                callback_type="legacy")
        dt = time.perf_counter() - t0
        # (digests: the 4096^2 fields would not fit the GPU box's output budget)
        res[name + "_x"] = np.frombuffer(hashlib.sha256(np.ascontiguousarray(x).tobytes()).digest(),
                                         dtype=np.uint8)
        res[name + "_hist"] = np.asarray(hist)
        res[name + "_its"] = np.array([K / dt])
        print(f"{tag} {name}: info {info}, {len(hist)} its, {K / dt:.1f} it/s", flush=True)
    np.savez(os.path.join(out_dir, f"ab_{tag}.npz"), **res)


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3])
        sys.exit(0)
    other, out_dir = sys.argv[1], sys.argv[2]
    os.makedirs(out_dir, exist_ok=True)
    for tag, lib in (("new", None), ("old", other), ("new2", None)):
        env = dict(os.environ)
        if lib:
            env["HH_LIB_PATH"] = lib
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", out_dir, tag],
                           env=env)
        if r.returncode != 0:
            sys.exit(r.returncode)
    a = np.load(os.path.join(out_dir, "ab_new.npz"))
    b = np.load(os.path.join(out_dir, "ab_old.npz"))
    c = np.load(os.path.join(out_dir, "ab_new2.npz"))
    bad = 0
    for name, *_ in CASES:
        same = all(np.array_equal(a[name + k], b[name + k]) for k in ("_x", "_hist"))
        bad += not same
        print(f"{name}: bit-identical {same}; it/s new {a[name + '_its'][0]:.1f} / "
              f"{c[name + '_its'][0]:.1f}, old {b[name + '_its'][0]:.1f}", flush=True)
    sys.exit(1 if bad else 0)
