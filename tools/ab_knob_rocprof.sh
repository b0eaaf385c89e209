#!/bin/bash
# A/B of one HH_* knob on the bench's GMRES: for each VALUE, rocprofv3 --kernel-trace --stats of
# `bench.py --no-cpu-baseline ARGS` with KNOB=VALUE, then the one-pass kernels' per-K TB/s
# (tools/fused_tbps.py) and the bench line's GMRES it/s.  Each run under its own time limit; a
# fault or time limit ends the session.
#   usage: tools/ab_knob_rocprof.sh OUTDIR KNOB "V1 V2 ..." [bench args...]
set -u
OUT=$1; KNOB=$2; VALS=$3; shift 3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
mkdir -p "$OUT"
for v in $VALS; do
  tag=$(basename "$v" | tr -c 'A-Za-z0-9\n' '_')
  d="$OUT/prof_${KNOB}_$tag"
  env "$KNOB=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/bench_${KNOB}_$tag.log" 2>&1
  rc=$?
  echo "== $KNOB=$v rc=$rc"
  case $rc in 0) ;; *) tail -5 "$OUT/bench_${KNOB}_$tag.log"; exit $rc;; esac
  stats=$(ls "$d"/*/run_kernel_stats.csv "$d"/run_kernel_stats.csv 2>/dev/null | head -1)
  python3 tools/fused_tbps.py "$stats" "${N:-4096}" 8 | tee "$OUT/tbps_${KNOB}_$tag.txt"
  grep '^{' "$OUT/bench_${KNOB}_$tag.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['gmres']; print('gmres it/s', g['iters_per_s'], g['solve_path'], g['final_rel_presid'], 'knobs', d['config'].get('knobs'))"
done
