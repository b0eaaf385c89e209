"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (separate runs, KB units) per kernel,
with the gfx950 correction from MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of a
16-B/lane coalesced read stream) and the algorithmic bytes of each kernel for comparison.
usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV [OUT_JSON]
"""
import csv
import json
import sys
from collections import defaultdict

N = 4096 * 4096
ALGO = {  # kernel-name fragment -> (read bytes, write bytes) per launch at 4096^2
    "p0(": (24 * N, 16 * N), "p1(": (24 * N, 16 * N), "p3(": (16 * N, 16 * N),
    "p4(": (24 * N, 0), "stencil_kernel<0": (24 * N, 16 * N), "tile_kernel<0": (24 * N, 16 * N),
}


def load(path):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


fetch, write = load(sys.argv[1]), load(sys.argv[2])
out = {}
for name in fetch:
    key = next((k for k in ALGO if k in name), None)
    if key is None:
        continue
    rd, wr = ALGO[key]
    f, w = fetch[name], write.get(name, float("nan"))
    out[key] = dict(kernel=name[:90], fetch_raw=f, write=w, fetch_x2=2 * f,
                    algo_read=rd, algo_write=wr,
                    read_ratio_x2=(2 * f / rd) if rd else None, write_ratio=(w / wr) if wr else None)
    print(f"{key:18s} FETCH raw {f/1e6:8.1f} MB (x2 {2*f/1e6:8.1f}) vs algo read {rd/1e6:7.1f} MB"
          f" | WRITE {w/1e6:7.1f} MB vs algo {wr/1e6:7.1f} MB")
if len(sys.argv) > 3:
    json.dump(out, open(sys.argv[3], "w"), indent=1)
