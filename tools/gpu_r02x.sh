#!/bin/bash
# Round-2 session X: wave-wide Givens column in the regular cycle (gmres_column_kernel /
# gmres_lag_kernel): bitwise A/B against the previous build, Krylov / distributed / config tests,
# config-2 and default bench lines.
set -u
TAG=${1:-r02x}
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
  echo "=== $name rc=$rc"; tail -8 "$OUT/$name.log" | cut -c1-500
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return $rc
}
PYT="python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu"
step ab 400 python tools/ab_lib_bits.py ab_prev/libhelmholtz_amd.so "$OUT/ab"
step t_kry 600 $PYT tests/test_gpu_small_cycle.py tests/test_gpu_gmres.py tests/test_gpu_krylov_modes.py tests/test_gpu_dist.py tests/test_gpu_configs.py tests/test_gpu_errors.py || exit 1
for fz in 0 3 1 2 0 3; do  # (HH_KRYLOV_FUSE bits: 1 multidot + reduce, 2 update + column)
  step bench_c2_fuse${fz}_$RANDOM 200 env HH_KRYLOV_FUSE=$fz python bench.py --config 2 --no-cpu-baseline
done
step prof_small 120 python tools/prof_small_cycle.py --iters 400
step bench 300 python bench.py --no-cpu-baseline
step rocprof 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --config 2 --no-cpu-baseline --gmres-iters 60
echo done
