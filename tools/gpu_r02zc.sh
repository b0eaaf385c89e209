#!/bin/bash
# Round-2 session ZC: batched partial loads in the column / reduce kernels: bitwise A/B against
# the previous build, Krylov tests, config-2 and default bench lines, rocprof of both.
set -u
TAG=${1:-r02zc}
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
  echo "=== $name rc=$rc"; tail -8 "$OUT/$name.log" | cut -c1-300
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return $rc
}
PYT="python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu"
step ab 400 python tools/ab_lib_bits.py ab_prev/libhelmholtz_amd.so "$OUT/ab"
rm -f "$OUT"/ab/*.npz
step t_kry 600 $PYT tests/test_gpu_gmres.py tests/test_gpu_krylov_modes.py tests/test_gpu_configs.py tests/test_gpu_spmv.py tests/test_gpu_variants.py || exit 1
step bench_c2a 200 python bench.py --config 2 --no-cpu-baseline
step bench_c2b 200 python bench.py --config 2 --no-cpu-baseline
step bench 300 python bench.py --no-cpu-baseline
step rocprof_c2 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv -- python3 bench.py --config 2 --no-cpu-baseline --gmres-iters 60
step rocprof 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --gmres-iters 40
echo done
