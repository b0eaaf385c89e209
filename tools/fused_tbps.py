"""TB/s of the one-pass GMRES kernels per K from a rocprofv3 kernel-stats CSV: a pass at
iteration K moves 16 (K + 3) B per unknown (+ 8 B of 1/c^2 for a non-constant medium; DESIGN
3g).  usage: python tools/fused_tbps.py STATS_CSV N [IC_BYTES]"""
import csv
import re
import sys

path, n = sys.argv[1], int(sys.argv[2])
ic = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
N = n * n
rows = []
with open(path) as fh:
    for r in csv.DictReader(fh):
        m = re.search(r"fused_(sl_iter|slk|slv|iter)_kernel<(\d+)", r["Name"])
        if m:
            K = int(m.group(2))
            ns = float(r["AverageNs"])
            gbs = (16 * (K + 3) + ic) * N / ns
            rows.append((K, "" if m.group(1) == "iter" else "_" + m.group(1), int(r["Calls"]),
                         ns / 1e3, gbs))
for K, sl, calls, us, gbs in sorted(rows):
    print(f"fused{sl}<{K:2d}>  calls {calls:5d}  avg {us:9.1f} us  {gbs / 1e3:5.2f} TB/s")
