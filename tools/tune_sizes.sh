#!/bin/bash
# Stencil shape x band height at several grid sizes / media (tools/tune_stencil.py per case).
# usage: tools/tune_sizes.sh TAG "n:medium n:medium ..." [variants] [rpbs] [rotate]
set -u
TAG=${1:-sizes}; CASES=${2:-"4096:const 8192:const 8192:marmousi 16384:const 16384:marmousi"}
VARS=${3:-42,30}; RPBS=${4:-16,32,64,128}; ROT=${5:-1}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for c in $CASES; do
  n=${c%%:*}; m=${c##*:}
  timeout -k 10 240 python tools/tune_stencil.py --n "$n" --medium "$m" --variants "$VARS" \
    --rpbs "$RPBS" --grids 0 --rounds 3 --rotate "$ROT" > "$OUT/tune_${m}_${n}_rot$ROT.log" 2>&1 || exit $?
  echo "== $n $m"; tail -n +5 "$OUT/tune_${m}_${n}_rot$ROT.log" | head -8
done
