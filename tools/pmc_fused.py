"""HBM traffic of the one-pass GMRES iteration (`fused_iter_kernel<K, ...>`) from two
rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs, KB units), per K, against its
algorithmic bytes: reads (K + 1) 16 B per unknown (the K basis vectors v_0 .. v_{K-1} and w_j),
writes 32 B (u_{j+1} into V[K], w_{j+1}); + 8 B read of 1/c^2 for a non-constant medium.
FETCH_SIZE is doubled (gfx950 correction for 16-B/lane coalesced reads, MI355X_MICROARCH.md),
as in tools/pmc_traffic.py.
usage: python tools/pmc_fused.py FETCH_CSV WRITE_CSV --n N [--rows R] [--medium const|marmousi]
       [--precond jacobi|sl|none] [--restart 20] [--knobs K=V,...] [--merge DB.json]
       (records the cycle's ratio and the per-K ratios under the key bench.py looks up,
       n{N}_rows{R}_{medium}_{precond}_r{restart}, with the kernel knobs the profiled run set;
       --rows: the slab height of one pass launch -- a virtual slab of the profiled run)"""
import argparse
import csv
import json
import os
import re
from collections import defaultdict


def load(path):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        m = re.search(r"fused_(sl_iter|slk|slv|iter)_kernel<(\d+)", r["Kernel_Name"])
        if m:
            tag = "" if m.group(1) == "iter" else "sl_"  # (every shifted-Laplace kernel: "sl")
            acc[(tag, int(m.group(2)))].append(float(r["Counter_Value"]) * 1024.0)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch")
    p.add_argument("write")
    p.add_argument("--n", type=int, required=True)
    p.add_argument("--medium", default="const")
    p.add_argument("--rows", type=int, default=0)
    p.add_argument("--precond", default="jacobi")
    p.add_argument("--restart", type=int, default=20)
    p.add_argument("--knobs", default="")
    p.add_argument("--merge")
    a = p.parse_args()
    rows = a.rows or a.n
    N = a.n * rows
    fetch, write = load(a.fetch), load(a.write)
    tot_t = tot_a = 0.0
    per_k = {}
    print(f"n={a.n} {a.medium}: per launch, MB (FETCH_SIZE x2 | WRITE_SIZE) vs algorithmic")
    for key in sorted(fetch):
        sl, K = key
        f, cnt = fetch[key]
        w = write.get(key, (float("nan"), 0))[0]
        rd = ((K + 1) * 16 + (0 if a.medium == "const" else 8)) * N
        wr = 32 * N
        tot_t += (2 * f + w) * cnt
        tot_a += (rd + wr) * cnt
        per_k[f"{'sl' if sl else ''}K{K}"] = round((2 * f + w) / (rd + wr), 4)
        print(f"{'sl ' if sl else ''}K={K:2d} x{cnt:3d}: read {2 * f / 1e6:9.1f} vs {rd / 1e6:9.1f} "
              f"({2 * f / rd:.3f}x, raw {f / rd:.3f}x) | write {w / 1e6:8.1f} vs {wr / 1e6:8.1f} "
              f"({w / wr:.3f}x) | total {(2 * f + w) / (rd + wr):.3f}x")
    if tot_a:
        print(f"all launches: {tot_t / 1e9:.2f} GB vs {tot_a / 1e9:.2f} GB algorithmic = "
              f"{tot_t / tot_a:.3f}x")
        if a.merge:
            key = f"n{a.n}_rows{rows}_{a.medium}_{a.precond}_r{a.restart}"
            knobs = dict(kv.split("=", 1) for kv in a.knobs.split(",") if kv)
            db = json.load(open(a.merge)) if os.path.exists(a.merge) else {}
            db[key] = {"ratio": round(tot_t / tot_a, 4), "per_K": per_k, "knobs": knobs,
                         "source": f"{os.path.basename(os.path.dirname(a.fetch))}, "
                                   f"{os.path.basename(os.path.dirname(a.write))}"}
            json.dump(db, open(a.merge, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
