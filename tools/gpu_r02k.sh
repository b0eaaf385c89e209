#!/bin/bash
# small-grid whole-cycle GMRES kernel: parity tests, then config 1 / 2 bench lines
set -u
TAG=${1:-r02k}
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
PYT="python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu"
step t_small 600 $PYT tests/test_gpu_small_cycle.py tests/test_gpu_errors.py tests/test_gpu_krylov_modes.py tests/test_gpu_gmres.py tests/test_gpu_driver.py tests/test_gpu_sweep.py tests/test_gpu_variants.py tests/test_gpu_configs.py -x
step prof_small 120 python tools/prof_small_cycle.py
step bench_c1 200 python bench.py --config 1 --no-cpu-baseline --steps 200
step rocprof_c1 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c1" -o run --output-format csv -- python3 tools/prof_small_cycle.py --iters 100
echo done
