"""The reference's own experiment, reproduced on the device.

code.py:558-611 (`__main__`) sweeps run_solver (code.py:424-541) over n in {127, 255, 511, 1023}
and the four media c1f1 / c1f2 / c2f1 / c2f2, each with its hand-tuned PML constant C (the
active c1f1 rows and the commented ones, code.py:574-592), and reports the init / solve split --
the only numbers the reference publishes (CS714_Project.pdf p.3-6).

For every row this runs, on the GPU, `helmholtz_preconditioner_amd.run_solver` with
  * "sweep-asis": exactly what run_solver runs (M x = algo2_4(f) for every x, the middle sweep
    u -= T u: quirks Q1/Q2) -- the reference's 1-3 callbacks and non-convergence;
  * "sweep": Engquist-Ying Alg. 2.4 with both quirks corrected,
and, on this box's host (up to --host-max-n), the oracle's SuperLU restatement of the same path
(oracle/helmholtz_oracle.py SweepState: algo2_3's splu factorisations, algo2_4's sweeps; scipy
gmres as code.py:516 calls it), timed the same way: init = media + assembly + algo2_3 (+ the
as-is path's algo2_4(f)), solve = the gmres call.  Iteration counts, exit codes and fields are
compared with the oracle's wherever the host runs it.  The CS714 figures are printed as context (other,
unspecified hardware).

usage: python tools/experiment_table.py [--host-max-n 511] [--rows all|c1f1] [--max-n 1023]
Test infrastructure: imports oracle/ as the checker and the host baseline only.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (n, wave_num, media, C): code.py:574-592, active (c1f1) and commented rows alike
ROWS = [(127, 16, "c1f1", 81), (127, 16, "c1f2", 61), (127, 16, "c2f1", 80), (127, 16, "c2f2", 84.2),
        (255, 32, "c1f1", 62), (255, 32, "c1f2", 61), (255, 32, "c2f1", 62), (255, 32, "c2f2", 100),
        (511, 64, "c1f1", 81), (511, 64, "c1f2", 62), (511, 64, "c2f1", 63.5), (511, 64, "c2f2", 85),
        (1023, 128, "c1f1", 100), (1023, 128, "c1f2", 100.6), (1023, 128, "c2f1", 100),
        (1023, 128, "c2f2", 100)]
# CS714_Project.pdf: (solve, init) seconds, unspecified hardware
CS714 = {(127, "c1f1"): (0.2, 1.6), (255, "c1f1"): (0.7, 1.9), (511, "c1f1"): (2.9, 7.2),
         (1023, "c1f1"): (13.6, 29.9), (1023, "c2f2"): (29.1, 30.1)}
B, ALPHA = 12, 2.0


def host_oracle(n, wn, media, C, corrected):
    """run_solver's path on the host: (init s, solve s, info, iterations, u)"""
    import helmholtz_preconditioner_amd as H
    from oracle import helmholtz_oracle as O
    t0 = time.time()
    omega, h, eta = O.problem_params(n, B, wn, ALPHA)
    c_mat, f_mat = getattr(H, f"init_{media[:2]}_{media[2:]}")(omega, n)
    f = f_mat.flatten()
    A = O.build_A_matrix(B, C, eta, omega, h, n, c_mat)
    M, _ = O.sweeping_preconditioner(B, C, eta, omega, h, n, c_mat, f=f, corrected=corrected)
    t1 = time.time()
    u, info, hist, _ = O.gmres_reference(A, f, M=M, rtol=1e-3)
    t2 = time.time()
    return t1 - t0, t2 - t1, int(info), len(hist), u


def main():
    p = argparse.ArgumentParser(description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--host-max-n", type=int, default=511)
    p.add_argument("--host-max-n-corrected", type=int, default=255,
                   help="host oracle of the corrected sweep (tens of SuperLU applies per solve)")
    p.add_argument("--rows", default="all", choices=["all", "c1f1"])
    p.add_argument("--max-n", type=int, default=1023)
    a = p.parse_args()
    import helmholtz_preconditioner_amd as H
    from bench import host_description
    print(f"host: {host_description()}", flush=True)
    rows = [r for r in ROWS if (a.rows == "all" or r[2] == "c1f1") and r[0] <= a.max_n]
    # warm-up (HIP initialisation, first launches) outside every timed row
    H.run_solver(63, B, 8, 61, ALPHA, H.init_c1_f1, False, verbose=False)
    hdr = ("| n | media | C | M | device init s | device solve s | its | info | host init s | "
           "host solve s | host its | host info | field vs host | CS714 solve / init s |")
    print(hdr)
    print("|" + "---|" * (hdr.count("|") - 1))
    for n, wn, media, C in rows:
        init = getattr(H, f"init_{media[:2]}_{media[2:]}")
        for pre in ("sweep-asis", "sweep"):
            ti, ts, det = H.run_solver(n, B, wn, C, ALPHA, init, False, preconditioner=pre,
                                       verbose=False, return_details=True)
            cells = [str(n), media, str(C), pre, f"{ti:.3f}", f"{ts:.3f}", str(det["iterations"]),
                     str(det["info"])]
            if n <= (a.host_max_n if pre == "sweep-asis" else a.host_max_n_corrected):
                hi, hs, hinfo, hits, hu = host_oracle(n, wn, media, C, pre == "sweep")
                du = np.linalg.norm(det["u"] - hu) / max(np.linalg.norm(hu), 1e-300)
                same = det["iterations"] == hits and int(det["info"]) == hinfo
                cells += [f"{hi:.2f}", f"{hs:.2f}", str(hits), str(hinfo),
                          f"{du:.1e}" + ("" if same else " (its/info differ)")]
            else:
                cells += ["-", "-", "-", "-", "-"]
            cs = CS714.get((n, media)) if pre == "sweep-asis" else None
            cells.append(f"{cs[0]} / {cs[1]}" if cs else "")
            print("| " + " | ".join(cells) + " |", flush=True)


if __name__ == "__main__":
    main()
