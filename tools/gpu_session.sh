#!/bin/bash
# One GPU-box session, parameterised: tools/gpu_session.sh TAG STEP [STEP ...]
# Every step runs under its own time limit; a fault / abort / time limit (rc 124 137 134 139)
# ends the session there, and so does a failing test step.  Outputs: gpurun_out/TAG/<step>.log
# (copy what is to be judged into profiles/).
#
# Steps (ARGS: comma-separated, passed on as separate arguments):
#   tests[:FILES]        python -m pytest -m gpu over tests/ or the listed test files
#   smoke                __graft_entry__.smoke()
#   bench[:ARGS]         python bench.py ARGS                  (log: bench<_args>.log)
#   driver               the driver's own command: bench.py --gpus 1 --steps 20 --warmup 5
#   configs              bench.py --config 1, 2, 4, 5 (config 3 is the default line)
#   rocprof[:ARGS]       rocprofv3 --kernel-trace --stats of bench.py --no-cpu-baseline ARGS, and
#                        the tile kernel's average over the timed launches
#   pmc[:ARGS]           FETCH_SIZE and WRITE_SIZE, one rocprofv3 --pmc pass each, of
#                        tools/prof_stencil.py ARGS (default --iters 20)
#   pmcset               the same at every BASELINE config's grid, summarised into pmc_traffic.json
#   pmcpy:SCRIPT[,ARGS]  FETCH_SIZE and WRITE_SIZE passes of python tools/SCRIPT ARGS
#   py:SCRIPT[,ARGS]     python tools/SCRIPT ARGS (diagnostics, tuning sweeps; limit PY_SECS, 420)
#   rocpy:SCRIPT[,ARGS]  the same under rocprofv3 --kernel-trace --stats
# example: tools/gpu_session.sh r03a tests smoke bench driver rocprof pmc
set -u
TAG=${1:?usage: tools/gpu_session.sh TAG STEP...}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
fatal() { case $1 in 124|137|134|139) return 0;; *) return 1;; esac; }
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T)): $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -6 "$OUT/$name.log" | cut -c1-400
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return $rc
}
slug() { echo "$1" | tr -c 'A-Za-z0-9\n' '_' | sed 's/__*/_/g; s/^_//; s/_$//'; }
PYT="python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu"
rocm-smi --showproductname > "$OUT/smi.log" 2>&1 || true
for st in "$@"; do
  kind=${st%%:*}; arg=""; [ "$kind" != "$st" ] && arg=${st#*:}
  IFS=',' read -r -a A <<< "$arg"
  case $kind in
    tests)   if [ -z "$arg" ]; then run tests 840 $PYT tests || exit 1
             else run "tests_$(slug "$arg")" 840 $PYT "${A[@]}" || exit 1; fi ;;
    smoke)   run smoke 150 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench)   run "bench${arg:+_$(slug "$arg")}" 420 python bench.py "${A[@]}" ;;
    driver)  run driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    configs) for c in 1 2 4 5; do run "bench_config$c" 300 python bench.py --config $c; done ;;
    rocprof) name="rocprof${arg:+_$(slug "$arg")}"
             run "$name" 300 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run \
               --output-format csv -- python3 bench.py --no-cpu-baseline "${A[@]}"
             python3 tools/rocprof_timed_avg.py "$OUT/$name/run_kernel_trace.csv" \
               "void hh::(anonymous namespace)::tile_kernel<0, false, 4" 200 \
               > "$OUT/${name}_timed.log" 2>&1 || true ;;
    pmc)     [ -z "$arg" ] && A=(--iters 20)
             name="pmc${arg:+_$(slug "$arg")}"
             run "${name}_fetch" 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/${name}_fetch" -o run \
               --output-format csv -- python3 tools/prof_stencil.py "${A[@]}"
             run "${name}_write" 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/${name}_write" -o run \
               --output-format csv -- python3 tools/prof_stencil.py "${A[@]}" ;;
    pmcset)  # FETCH / WRITE passes of the apply at every BASELINE config's grid (+ 9-point),
             # merged into $OUT/pmc_traffic.json (bench.py reads profiles/r03_pmc_traffic.json)
             for cfg in 128:const:5 1024:const:5 4096:marmousi:5 4096:const:5 4096:marmousi:9 \
                        8192:const:5 16384:const:5; do
               IFS=':' read -r pn pm ps <<< "$cfg"
               it=20; [ "$pn" -le 1024 ] && it=200
               nm="pmcset_${pn}_${pm}_s${ps}"
               for ctr in FETCH_SIZE WRITE_SIZE; do
                 run "${nm}_$ctr" 240 rocprofv3 --pmc $ctr -d "$OUT/${nm}_$ctr" -o run \
                   --output-format csv -- python3 tools/prof_stencil.py --n "$pn" --medium "$pm" \
                   --stencil "$ps" --iters $it
               done
               python3 tools/pmc_traffic.py "$OUT/${nm}_FETCH_SIZE/run_counter_collection.csv" \
                 "$OUT/${nm}_WRITE_SIZE/run_counter_collection.csv" --n "$pn" --medium "$pm" \
                 --stencil "$ps" --merge "$OUT/pmc_traffic.json" || true
             done ;;
    pmcpy)   # FETCH_SIZE / WRITE_SIZE passes (one rocprofv3 --pmc run each) of tools/SCRIPT ARGS
             name="pmcpy_$(slug "$arg")"
             for ctr in FETCH_SIZE WRITE_SIZE; do
               run "${name}_$ctr" 300 rocprofv3 --pmc $ctr -d "$OUT/${name}_$ctr" -o run \
                 --output-format csv -- python3 "tools/${A[0]}" "${A[@]:1}"
             done ;;
    py)      run "py_$(slug "$arg")" "${PY_SECS:-420}" python "tools/${A[0]}" "${A[@]:1}" ;;
    rocpy)   name="rocpy_$(slug "$arg")"
             run "$name" 420 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run \
               --output-format csv -- python3 "tools/${A[0]}" "${A[@]:1}" ;;
    *)       echo "unknown step '$st'"; exit 2 ;;
  esac
done
echo done
