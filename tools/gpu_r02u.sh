#!/bin/bash
# Round-2 session U: small-cycle Givens wave (parallel column, readlane rotations, reciprocal
# solve): parity tests, phase profile, config-1 bench; 9-point fused M A v2 inside SL-GMRES
# (rocprof kernel stats of the 9-point bench line).
set -u
TAG=${1:-r02u}
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
  echo "=== $name rc=$rc"; tail -4 "$OUT/$name.log" | cut -c1-500
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return $rc
}
PYT="python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu"
step t_small 400 $PYT tests/test_gpu_small_cycle.py tests/test_gpu_gmres.py tests/test_gpu_krylov_modes.py tests/test_gpu_errors.py tests/test_gpu_driver.py || exit 1
step prof_small 120 python tools/prof_small_cycle.py --iters 400
step prof_small_jac 120 python tools/prof_small_cycle.py --iters 400 --precond jacobi
step bench_c1 200 python bench.py --config 1 --no-cpu-baseline --steps 200
step rocprof9 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof9" -o run --output-format csv -- python3 bench.py --stencil 9 --no-cpu-baseline --gmres-iters 40
echo done
