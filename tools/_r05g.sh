set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05g; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
for cfg in "4096 100 sl marmousi" "1024 64 jacobi const" "8192 256 jacobi const"; do
  set -- $cfg; n=$1; wn=$2; pc=$3; med=$4
  for ctr in FETCH_SIZE WRITE_SIZE; do
    PRECOND=$pc MODES=fused timeout -s KILL 300 rocprofv3 --pmc $ctr -d $O/pmc_${n}_$ctr -o run --output-format csv -- python3 tools/ab_krylov_mode.py $n $wn 1 > $O/pmc_${n}_$ctr.log 2>&1; rc=$?; echo "pmc $n $ctr rc=$rc"; fatal $rc pmc
  done
  python3 tools/pmc_fused.py $O/pmc_${n}_FETCH_SIZE/run_counter_collection.csv $O/pmc_${n}_WRITE_SIZE/run_counter_collection.csv --n $n --medium $med --precond $pc --restart 20 --merge $O/r05_pmc_fused.json | tee $O/pmc_${n}.txt
done
