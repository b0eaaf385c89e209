#!/bin/bash
# sweeping preconditioner: parity tests, then apply timings (persistent chain vs one launch
# per GEMV)
set -u
TAG=${1:-r02sw}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
fatal() { case $1 in 124|137|134|139) return 0;; *) return 1;; esac; }
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -8 "$OUT/$name.log" | cut -c1-600
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu"
step t_sweep 500 $PYT tests/test_gpu_sweep.py -x
step bench_chain 300 python tools/bench_sweep.py --form dense 127 255 511 1023
HH_SWEEP_CHAIN=0 step bench_launches 300 python tools/bench_sweep.py --form dense 127 255 511 1023
echo done
