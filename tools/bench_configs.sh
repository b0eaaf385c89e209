#!/bin/bash
# BASELINE.json configs 1, 2, 4, 5 as single-GPU bench lines (config 3 is the default bench),
# plus a stencil-shape sweep on the constant-medium (32 B/point) kernel.
# usage: tools/bench_configs.sh TAG
set -u
TAG=${1:-cfg}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for c in 1 2 4 5; do
  timeout -k 10 240 python bench.py --config $c > "$OUT/bench_config$c.log" 2>&1 || exit $?
  tail -c 400 "$OUT/bench_config$c.log"; echo
done
timeout -k 10 300 python tools/tune_stencil.py --n 8192 --medium const --variants 42,30,18,45 \
  --rpbs 16,32,64 --grids 0 --rounds 2 > "$OUT/tune_const8192.log" 2>&1 || exit $?
tail -14 "$OUT/tune_const8192.log"
