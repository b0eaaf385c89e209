"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (separate runs, KB units) of the operator
apply kernels, with the gfx950 correction from MI355X_MICROARCH.md (FETCH_SIZE counts half the
bytes of a 16-B/lane coalesced read stream: doubled) next to each kernel's algorithmic bytes
(read u 16 + 1/c^2 8, write y 16 per unknown; 16 + 16 for a constant medium).

usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV --n N --medium M [--stencil S]
                                   [--rows R] [--merge OUT_JSON]
--merge adds the record under key "n{N}_rows{R}_{M}_s{S}" to OUT_JSON (bench.py's
measured_traffic reads profiles/r05_pmc_traffic.json); --rows: the rows of one apply launch (a
virtual slab of the profiled run, tools/prof_stencil.py --virtual-slabs; default the grid).
"""
import argparse
import csv
import json
import os
from collections import defaultdict

KERNELS = ("tile_kernel<0", "tile9_kernel<0", "stencil_kernel<0")  # the EPI_AX apply kernels


def load(path):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch")
    p.add_argument("write")
    p.add_argument("--n", type=int, required=True)
    p.add_argument("--medium", default="marmousi")
    p.add_argument("--stencil", type=int, default=5)
    p.add_argument("--rows", type=int, default=0)
    p.add_argument("--merge")
    a = p.parse_args()
    rows = a.rows or a.n
    N = a.n * rows
    rd = (16 if a.medium == "const" else 24) * N
    wr = 16 * N
    fetch, write = load(a.fetch), load(a.write)
    rec = None
    for name, (f, cnt) in sorted(fetch.items(), key=lambda kv: -kv[1][1]):
        if not any(k in name for k in KERNELS):
            continue
        w = write.get(name, (float("nan"), 0))[0]
        rec = dict(kernel=name[:110], launches=cnt, fetch_raw=f, fetch_x2=2 * f, write=w,
                   algo_read=rd, algo_write=wr, traffic=2 * f + w,
                   ratio=(2 * f + w) / (rd + wr), read_ratio_x2=2 * f / rd, write_ratio=w / wr)
        print(f"n={a.n} {a.medium} s{a.stencil} {name[:70]}: FETCH x2 {2 * f / 1e6:9.1f} MB vs "
              f"algo read {rd / 1e6:9.1f} | WRITE {w / 1e6:9.1f} vs {wr / 1e6:9.1f} | total "
              f"{rec['ratio']:.3f}x algorithmic ({cnt} launches)")
        break  # the apply kernel with the most launches (the timed ones)
    if rec and a.merge:
        db = json.load(open(a.merge)) if os.path.exists(a.merge) else {}
        db[f"n{a.n}_rows{rows}_{a.medium}_s{a.stencil}"] = rec
        json.dump(db, open(a.merge, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
