#!/bin/bash
# Round-2 closing session, part A (PART=a): full GPU suite, smoke, the bench line as the driver
# runs it (--steps 20 --warmup 5) and with the defaults; part B (PART=b): BASELINE configs 1/2/4/5,
# rocprofv3 kernel trace of the default bench + timed-launch average, PMC traffic passes, the
# 9-point line, the sweeping apply bench.
set -u
TAG=${1:-r02final}
PART=${PART:-a}
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
  echo "=== $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-400
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
if [ "$PART" = c ]; then  # Krylov re-check: GMRES/Krylov tests, bench, rocprof of the bench
  step t_krylov 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gmres.py tests/test_gpu_krylov_modes.py tests/test_gpu_configs.py
  step bench 300 python bench.py
  step bench_config4 240 python bench.py --config 4 --no-cpu-baseline
  step rocprof 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --gmres-iters 40
elif [ "$PART" = a ]; then
  step t_all 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests
  step smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
  step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
  step bench 300 python bench.py
else
  step t_krylov 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gmres.py tests/test_gpu_krylov_modes.py tests/test_gpu_configs.py
  for c in 1 2 4 5; do step bench_config$c 240 python bench.py --config $c --no-cpu-baseline; done
  step rocprof 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --gmres-iters 40
  python3 tools/rocprof_timed_avg.py "$OUT/prof/run_kernel_trace.csv" "void hh::(anonymous namespace)::tile_kernel<0, false, 4" 200 > "$OUT/rocprof_timed.log" 2>&1 || true
  step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 tools/prof_stencil.py --iters 20
  step pmc_write 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 tools/prof_stencil.py --iters 20
  step bench9 240 python bench.py --stencil 9 --no-cpu-baseline
  step sweep 300 python tools/bench_sweep.py --form dense 127 255 511 1023
fi
echo done
