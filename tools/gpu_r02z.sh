#!/bin/bash
# small-cycle host-side costs: sync mode x callback
set -u
TAG=${1:-r02z}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for m in 0 1 2; do
  for cb in lambda none; do
    echo "== sync $m cb $cb"
    HH_SYNC_MODE=$m timeout -k 10 120 python tools/prof_small_cycle.py --cb $cb --iters 400 > "$OUT/p_${m}_${cb}.log" 2>&1 || { echo "rc=$?"; cat "$OUT/p_${m}_${cb}.log"; exit 1; }
    cat "$OUT/p_${m}_${cb}.log" | cut -c1-80
  done
done
