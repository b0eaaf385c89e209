#!/bin/bash
# the bench line as the driver runs it (--steps 20 --warmup 5) and with the defaults
set -u
TAG=${1:-r02bench}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || exit $?
for f in bench_driver bench; do
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$f.log') if l.startswith('{')][-1]); print('$f', d['value'], d['pct_hbm_peak'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['gmres']['iters_per_s'], d['spmv_constant_medium']['value'])"
done
