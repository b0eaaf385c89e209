#!/bin/bash
# One GPU-box session: parity tests, a bench line, and a rocprofv3 kernel-trace profile.
# Every GPU step has its own time limit; a fault/abort/timeout stops the session.
# usage: tools/gpu_session.sh TAG [pytest-args...]
set -u
TAG=${1:-r01}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
fatal() { case $1 in 124|137|134|139|-6|-11) return 0;; *) return 1;; esac; }
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
rocm-smi --showproductname > "$OUT/smi.log" 2>&1 || true
step pytest_gpu 480 python -m pytest tests -m gpu -q -x "$@"
step smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
step rocprof 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --gmres-iters 40
python3 tools/rocprof_timed_avg.py "$OUT/prof/run_kernel_trace.csv" "void hh::(anonymous namespace)::tile_kernel<0, false, 4" 200 > "$OUT/rocprof_timed.log" 2>&1 || true
step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 tools/prof_stencil.py --iters 20
step pmc_write 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 tools/prof_stencil.py --iters 20
step bench9 300 python bench.py --stencil 9
step rocprof9 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof9" -o run --output-format csv -- python3 bench.py --stencil 9 --no-cpu-baseline --gmres-iters 40
step pmc_fetch9 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch9" -o run --output-format csv -- python3 tools/prof_stencil.py --iters 20 --stencil 9
step pmc_write9 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write9" -o run --output-format csv -- python3 tools/prof_stencil.py --iters 20 --stencil 9
step sweep 300 python tools/bench_sweep.py --form dense 127 255 511 1023
step sweep_thomas 200 python tools/bench_sweep.py --form thomas 127 255
step export 200 python tools/bench_export.py
HH_SWEEP_GRAPH=0 step rocprof_sweep 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof_sweep" -o run --output-format csv -- python3 tools/bench_sweep.py --form dense 1023
echo done
