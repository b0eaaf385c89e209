set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05w; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
# the one-pass Jacobi passes at 16384^2 (config 5): PMC per K, for the bench line's pass traffic
for ctr in FETCH_SIZE WRITE_SIZE; do
  PRECOND=jacobi MODES=fused timeout -s KILL 400 rocprofv3 --pmc $ctr -d $O/pmc_16384_$ctr -o run --output-format csv -- python3 tools/ab_krylov_mode.py 16384 512 1 > $O/pmc_16384_$ctr.log 2>&1; rc=$?; echo "pmc $ctr rc=$rc"; fatal $rc pmc
done
python3 tools/pmc_fused.py $O/pmc_16384_FETCH_SIZE/run_counter_collection.csv $O/pmc_16384_WRITE_SIZE/run_counter_collection.csv --n 16384 --medium const --precond jacobi --restart 20 --merge $O/r05_pmc_fused.json | tail -4
