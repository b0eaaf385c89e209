#!/bin/bash
# sweep chain timing variants (HH_SWEEP_DIAG: low bits 1 no matrix loads, 2 no input waits,
# 3 neither loads nor input reads, 4 no input reads -- wrong results, timing only; +16 a third
# barrier per step) and the launch-per-GEMV form
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r02sd
HH_SWEEP_CHAIN=1 timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sweep.py > gpurun_out/r02sd/t_sweep.log 2>&1; rc=$?
tail -2 gpurun_out/r02sd/t_sweep.log; [ $rc -eq 0 ] || exit $rc
for d in ${DIAGS:-0 32 0 32}; do
  echo "== chain diag $d"
  HH_SWEEP_CHAIN=1 HH_SWEEP_DIAG=$d timeout -k 10 120 python tools/bench_sweep.py --form dense 1023 2>&1 | cut -c1-100 || exit 1
done
echo "== launches"
HH_SWEEP_CHAIN=0 timeout -k 10 120 python tools/bench_sweep.py --form dense 1023 2>&1 | cut -c1-100
