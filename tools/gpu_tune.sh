#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tune}; mkdir -p "$OUT"; shift || true
timeout -k 10 400 python tools/tune_stencil.py "$@" > "$OUT/tune.log" 2>&1; rc=$?
cat "$OUT/tune.log" | tail -45; exit $rc
