#!/bin/bash
# Round-2 session B: bit-identity of the new fused shifted-Laplace shapes, then their timing.
set -u
TAG=${1:-r02b}
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
  echo "=== $name rc=$rc"; tail -12 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu"
step t_shapes 300 $PYT tests/test_gpu_variants.py -k "shapes_bit_identical" -x
step t_errors 200 $PYT tests/test_gpu_errors.py -k default_maxiter
step t_fused 300 $PYT tests/test_gpu_variants.py -k "shapes_bit" -x
step tune_sl2 300 python tools/tune_sl2.py --variants 165,163,167,171,175 --rpbs 16,32 --rounds 3
step tune_sl2_gmres 300 python tools/tune_gmres_variant.py 4096 -1,167,175
echo done
