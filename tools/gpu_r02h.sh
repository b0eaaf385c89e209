#!/bin/bash
# one-allreduce GMRES: single-rank parity, multi-rank (default lagged) parity, timing
set -u
TAG=${1:-r02h}
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
  echo "=== $name rc=$rc"; tail -6 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu"
step t_gmres 300 $PYT tests/test_gpu_gmres.py tests/test_gpu_driver.py
step t_dist 600 $PYT tests/test_gpu_dist.py tests/test_gpu_configs.py -k "not config2 and not config3"
echo done
