#!/bin/bash
# Round-2 session PMC: HBM traffic of the fused shifted-Laplace M A and the Krylov kernels inside
# one SL-GMRES(20) cycle at 4096^2 (FETCH_SIZE / WRITE_SIZE in separate passes), and the
# small-grid cycle kernel's duration per cycle (config 1) from a kernel trace.
set -u
TAG=${1:-r02pmc}
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
step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 tools/prof_stencil.py --iters 5 --gmres
step pmc_write 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 tools/prof_stencil.py --iters 5 --gmres
step trace_c1 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c1" -o run --output-format csv -- python3 tools/prof_small_cycle.py --iters 400
echo done
