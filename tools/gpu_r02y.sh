#!/bin/bash
# Round-2 session Y: small-cycle reducer on one wave (DPP sums): parity tests, profile, config 1
set -u
TAG=${1:-r02y}
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
  echo "=== $name rc=$rc"; tail -8 "$OUT/$name.log" | cut -c1-400
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return $rc
}
PYT="python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu"
step t_small 500 $PYT tests/test_gpu_small_cycle.py tests/test_gpu_gmres.py tests/test_gpu_sweep.py tests/test_gpu_driver.py || exit 1
step prof_small 120 python tools/prof_small_cycle.py --iters 400
step bench_c1 200 python bench.py --config 1 --no-cpu-baseline --steps 200
step prof_small2 120 python tools/prof_small_cycle.py --iters 400
echo done
