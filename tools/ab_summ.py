"""Filter for tools/ab_env.sh: prints a bench.py JSON line's SpMV value and GMRES rates, or any
"it/s" line, prefixed by the A/B setting given as argv[1]."""
import json
import sys

tag = sys.argv[1]
for line in sys.stdin:
    line = line.rstrip()
    if line.startswith("{"):
        d = json.loads(line)
        g = d.get("gmres") or {}
        print("[%s] spmv %s GB/s  gmres %s it/s  pass %s GB/s  path %s"
              % (tag, d.get("value"), g.get("iters_per_s"), g.get("pass_GBps"),
                 g.get("solve_path")))
    elif "it/s" in line:
        print("[%s] %s" % (tag, line[:300]))
