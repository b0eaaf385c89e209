#!/bin/bash
# Full GPU suite + smoke + default bench line (after a default kernel change).
set -u
TAG=${1:-r02g}
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
  echo "=== $name rc=$rc"; tail -4 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
step t_all 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests
step smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
echo done
