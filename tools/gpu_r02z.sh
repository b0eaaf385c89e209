#!/bin/bash
# Round-2 session Z: small-cycle block width A/B (1, 2, 4 copies of the row's threads), config 1
set -u
TAG=${1:-r02z}
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
  echo "=== $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-300
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return $rc
}
for w in 4 1 2 4 1 2; do
  step prof_w${w}_$RANDOM 120 env HH_SMALL_WIDE=$w python tools/prof_small_cycle.py --iters 400
done
echo done
