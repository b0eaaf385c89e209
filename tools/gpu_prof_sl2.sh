#!/bin/bash
# rocprofv3 kernel stats of the fused shifted-Laplace M A inside GMRES(20) at the bench workload,
# one profiled process per (variant, band height); prints the sl2_kernel line of each.
# usage: tools/gpu_prof_sl2.sh TAG "V:R V:R ..."
set -u
TAG=${1:-sl2prof}; SHAPES=${2:-"-1:0 175:0 175:16"}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for vr in $SHAPES; do
  V=${vr%%:*}; R=${vr##*:}
  D="$OUT/p_${V}_${R}"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$D" -o run --output-format csv -- \
    python3 tools/prof_stencil.py --iters 1 --gmres --variant "$V" --rpb "$R" > "$D.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rocprof $V:$R rc=$rc"; tail -5 "$D.log"; exit $rc; }
  f=$(find "$D" -name '*kernel_stats.csv' | head -1)
  echo "variant $V rpb $R: $(grep -h 'sl2_kernel' "$f" | cut -c1-220)"
done
