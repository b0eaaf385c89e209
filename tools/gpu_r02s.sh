#!/bin/bash
# Round-2 session S: small-cycle wide-block A/B (config 1), then the full GPU suite, smoke and the
# bench line as the driver runs it and with the defaults.
set -u
TAG=${1:-r02s}
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
step prof_wide 120 python tools/prof_small_cycle.py --iters 400
step prof_narrow 120 env HH_SMALL_WIDE=0 python tools/prof_small_cycle.py --iters 400
step bench_c1 200 python bench.py --config 1 --no-cpu-baseline --steps 200
step bench_c1_narrow 200 env HH_SMALL_WIDE=0 python bench.py --config 1 --no-cpu-baseline --steps 200
[ "${FULL:-1}" = 1 ] || { echo done; exit 0; }
step t_all 900 $PYT tests
step smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench 300 python bench.py
echo done
