set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05l; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_krylov_modes.py tests/test_gpu_gmres.py tests/test_gpu_configs.py tests/test_gpu_small_cycle.py tests/test_gpu_dist.py tests/test_gpu_variants.py > $O/tests_k.log 2>&1; rc=$?; echo "tests_k rc=$rc"; tail -3 $O/tests_k.log; fatal $rc tests_k
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh 3 "HH_LAG_RED=0" "HH_LAG_RED=1" -- python bench.py --config 2 --no-cpu-baseline > $O/ab_lagred.log 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/ab_lagred.log; fatal $rc ab
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_c2 -o run --output-format csv -- python3 bench.py --config 2 --no-cpu-baseline > $O/rocprof_c2.log 2>&1; rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
grep -E "cycle_coef|lag_red|gmres_lag|reduce_kernel|gmres_solve|cycle_end|cycle_finish" $O/rocprof_c2/run_kernel_stats.csv | cut -c1-200
