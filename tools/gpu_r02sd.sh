#!/bin/bash
# sweep chain diagnostics: full, no matrix loads, no input waits (wrong results, timing only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r02sd
export HH_SWEEP_CHAIN=1
for d in 0 1 2; do
  echo "== diag $d"
  HH_SWEEP_DIAG=$d timeout -k 10 120 python tools/bench_sweep.py --form dense 127 1023 2>&1 | grep -v SuperLU | cut -c1-110 || exit 1
done
