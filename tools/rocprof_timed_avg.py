"""Average duration of one kernel over its last K launches in a rocprofv3 kernel trace -- the
timed region of bench.py (its warm-up launches come first), to set beside the bench line's
HIP-event kernel_ms.  usage: rocprof_timed_avg.py TRACE.csv KERNEL_PREFIX K"""
import csv
import statistics
import sys

path, prefix, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].startswith(prefix)]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print(f"{prefix}: {len(d)} launches; all: avg {sum(d) / len(d):.2f} us; first {len(d) - k}: avg "
      f"{sum(d[:-k]) / max(1, len(d) - k):.2f} us; last {k} (timed): avg {sum(d[-k:]) / k:.2f} us, "
      f"median {statistics.median(d[-k:]):.2f} us, min {min(d[-k:]):.2f} us")
