"""Interleaved A/B of bench.py lines across builds / environment knobs on one box.

usage: python tools/ab_bench.py --rounds 3 --args "--config 2 --no-cpu-baseline" \
           --variant new= --variant r02=HH_LIB_PATH=ab_prev/libhelmholtz_amd_r02.so,HH_LIB_AB=1
Each variant is NAME=ENV1=V1,ENV2=V2 (empty: the tree as is).  Prints per run the SpMV value
and GMRES it/s, then the per-variant medians.  Diagnostic only.
"""
import argparse
import json
import os
import shlex
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--args", default="--no-cpu-baseline")
    p.add_argument("--variant", action="append", required=True)
    a = p.parse_args()
    variants = []
    for v in a.variant:
        name, _, env = v.partition("=")
        kv = dict(e.split("=", 1) for e in env.split(",") if e)
        variants.append((name, kv))
    res = {n: [] for n, _ in variants}
    for r in range(a.rounds):
        for name, kv in variants:
            env = dict(os.environ, **kv)
            out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] +
                                 shlex.split(a.args), env=env, capture_output=True, text=True,
                                 timeout=600, cwd=ROOT)
            line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
            if out.returncode != 0 or not line:
                print(f"{name} round {r}: FAILED rc={out.returncode}\n{out.stderr[-2000:]}",
                      flush=True)
                sys.exit(1)
            d = json.loads(line[-1])
            g = (d.get("gmres") or {}).get("iters_per_s")
            res[name].append((d["value"], g))
            print(f"{name:10s} round {r}: spmv {d['value']:9.2f} GB/s  kernel "
                  f"{d['roofline']['kernel_ms'] * 1e3:8.2f} us  gmres {g} it/s", flush=True)
    for name, vals in res.items():
        gs = [g for _, g in vals if g]
        print(f"{name:10s} median spmv {statistics.median(v for v, _ in vals):9.2f} GB/s  "
              f"gmres {statistics.median(gs) if gs else None} it/s")


if __name__ == "__main__":
    main()
