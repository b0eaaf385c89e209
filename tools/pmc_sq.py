"""Where a kernel's waves spend their cycles, from one rocprofv3 --pmc pass of SQ counters
(MI355X_MICROARCH.md 'rocprofv3 PMC slots': SQ_WAIT_ANY = parked on s_waitcnt / barrier,
SQ_WAIT_INST_ANY = issue stalls, SQ_ACTIVE_INST_ANY = issuing; together ~ SQ_WAVE_CYCLES),
per kernel name (one line per template instance), summed over its launches.
usage: python tools/pmc_sq.py COUNTER_CSV [--match REGEX]"""
import argparse
import csv
import re
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("csv")
    p.add_argument("--match", default="fused")
    a = p.parse_args()
    acc = defaultdict(lambda: defaultdict(float))
    launches = defaultdict(set)
    for r in csv.DictReader(open(a.csv)):
        name = r["Kernel_Name"]
        if not re.search(a.match, name):
            continue
        short = re.sub(r"\(.*", "", name.replace("void hh::(anonymous namespace)::", ""))
        acc[short][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[short].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    print(f"{'kernel':42s} {'launch':>6s} {'wave_cyc':>10s} {'active':>7s} {'wait':>7s} "
          f"{'instst':>7s} {'valu/w':>8s} {'salu/w':>8s} {'lds_st':>7s}")
    for k in sorted(acc, key=lambda s: (re.sub(r"<.*", "", s), int((re.findall(r"<(\d+)", s) or [0])[0]))):
        c = acc[k]
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        waves = c.get("SQ_WAVES", 0.0) or 1.0
        print(f"{k[:42]:42s} {len(launches[k]):6d} {wc / len(launches[k]):10.3g} "
              f"{c.get('SQ_ACTIVE_INST_ANY', 0) / wc:7.3f} {c.get('SQ_WAIT_ANY', 0) / wc:7.3f} "
              f"{c.get('SQ_WAIT_INST_ANY', 0) / wc:7.3f} {c.get('SQ_INSTS_VALU', 0) / waves:8.0f} "
              f"{c.get('SQ_INSTS_SALU', 0) / waves:8.0f} {c.get('SQ_WAIT_INST_LDS', 0) / wc:7.3f}")


if __name__ == "__main__":
    main()
