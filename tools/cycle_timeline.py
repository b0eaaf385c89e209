"""One GMRES restart cycle's GPU timeline from a rocprofv3 kernel trace: every launch between two
gmres_start_kernel launches (the last full cycle of the trace), its duration and the idle gap
before it, and the cycle's span / busy / idle totals -- where a cycle's time goes besides the
passes (host round trips show as gaps before the first kernels after a sync).
usage: python tools/cycle_timeline.py RUN_kernel_trace.csv [--all]
       (--all prints every launch; default: only the non-pass kernels and gaps > 3 us)"""
import csv
import sys


def main():
    path = sys.argv[1]
    show_all = "--all" in sys.argv
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "gmres_start_kernel" in r["Kernel_Name"]]
    if len(starts) < 2:
        sys.exit("fewer than two gmres_start_kernel launches in the trace")
    seg = rows[starts[-2]:starts[-1]]
    t0 = int(seg[0]["Start_Timestamp"])
    prev, busy, idle = None, 0, 0
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = s - prev if prev is not None else 0
        busy += e - s
        idle += max(gap, 0)
        name = r["Kernel_Name"].replace("hh::(anonymous namespace)::", "").replace("void ", "")
        hot = "fused_" in name or "lag_red" in name
        if show_all or not hot or gap > 3000:
            print(f"{(s - t0) / 1e3:9.2f} us  {(e - s) / 1e3:8.2f} us  gap {gap / 1e3:7.2f}  "
                  f"{name[:70]}")
        prev = e
    span = int(rows[starts[-1]]["Start_Timestamp"]) - t0
    print(f"cycle: {len(seg)} launches, span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us, "
          f"idle {idle / 1e3:.1f} us")


if __name__ == "__main__":
    main()
