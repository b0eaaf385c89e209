# PMC (FETCH_SIZE x2 + WRITE_SIZE, one rocprofv3 --pmc pass each) of the apply and of the
# one-pass GMRES passes at the per-rank slab shapes the driver's N-GPU bench runs (VERDICT r04
# item 6), each rank's slab emulated as a virtual slab of one process on one GPU, merged into
# $OUT/r05_pmc_traffic.json (apply) and $OUT/r05_pmc_fused.json (passes): the records
# bench.py's roofline.traffic and gmres.pass_traffic_vs_algorithmic look up by (n, slab rows).
#   tools/pmc_shapes.sh [SHAPES...]   SHAPE = n:slabs, default: the weak-scaling grids of N = 1,
#   2, 4, 8 (4096:1 5792:2 8192:4 11584:8) and the same-N 4096^2 legs (4096:2 4096:4 4096:8)
# Env: KNOBS (comma list recorded with the pass records, e.g. HH_SLK=1) -- also exported;
# PASSES_ONLY=1 skips the apply records (the one-pass kernels changed, the apply did not);
# APPLY_ONLY=1 the pass records.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_shapes}; mkdir -p $OUT
KNOBS=${KNOBS:-}
for kv in ${KNOBS//,/ }; do export "$kv"; done
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
SHAPES=("$@"); [ ${#SHAPES[@]} -eq 0 ] && SHAPES=(4096:1 5792:2 8192:4 11584:8 4096:2 4096:4 4096:8)
for sh in "${SHAPES[@]}"; do
  n=${sh%%:*}; s=${sh##*:}; rows=$((n / s))
  for med in $([ "${PASSES_ONLY:-0}" = 1 ] || echo marmousi const); do
    nm="apply_${n}_${s}_${med}"
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 300 rocprofv3 --pmc $ctr -d $OUT/${nm}_$ctr -o run --output-format csv -- \
        python3 tools/prof_stencil.py --n $n --medium $med --iters 20 --virtual-slabs $s \
        > $OUT/${nm}_$ctr.log 2>&1; rc=$?; fatal $rc $nm; [ $rc -ne 0 ] && { tail -5 $OUT/${nm}_$ctr.log; exit $rc; }
    done
    python3 tools/pmc_traffic.py $OUT/${nm}_FETCH_SIZE/run_counter_collection.csv \
      $OUT/${nm}_WRITE_SIZE/run_counter_collection.csv --n $n --medium $med --rows $rows \
      --merge $OUT/r05_pmc_traffic.json || true
  done
  [ "${APPLY_ONLY:-0}" = 1 ] && continue
  nm="pass_${n}_${s}_sl"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    PRECOND=sl MODES=fused VSLABS=$s timeout -k 10 400 rocprofv3 --pmc $ctr -d $OUT/${nm}_$ctr -o run \
      --output-format csv -- python3 tools/ab_krylov_mode.py $n 100 1 > $OUT/${nm}_$ctr.log 2>&1
    rc=$?; fatal $rc $nm; [ $rc -ne 0 ] && { tail -5 $OUT/${nm}_$ctr.log; exit $rc; }
  done
  python3 tools/pmc_fused.py $OUT/${nm}_FETCH_SIZE/run_counter_collection.csv \
    $OUT/${nm}_WRITE_SIZE/run_counter_collection.csv --n $n --rows $rows --medium marmousi \
    --precond sl --restart 20 --knobs "$KNOBS" --merge $OUT/r05_pmc_fused.json | tail -3 || true
done
echo done
