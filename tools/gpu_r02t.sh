#!/bin/bash
# Round-2 session T: small-cycle Givens wave (config 1) and the 9-point fused M A v2 shape:
# parity tests, phase profile, shape tuning, bench lines.
set -u
TAG=${1:-r02t}
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
step t_small 400 $PYT tests/test_gpu_small_cycle.py tests/test_gpu_gmres.py tests/test_gpu_krylov_modes.py || exit 1
step prof_small 120 python tools/prof_small_cycle.py --iters 400
step bench_c1 200 python bench.py --config 1 --no-cpu-baseline --steps 200
step t_s9 400 $PYT tests/test_gpu_variants.py tests/test_gpu_stencil9.py -k "shifted_laplace or stencil9 or shapes" || exit 1
step tune_s9 300 python tools/tune_sl2.py --stencil 9 --variants 160,164,163,167,171,175 --rpbs 16,32,60 --rounds 2
step bench9 240 python bench.py --stencil 9 --no-cpu-baseline
echo done
