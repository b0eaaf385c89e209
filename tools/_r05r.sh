set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05r; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_krylov_modes.py tests/test_gpu_configs.py tests/test_gpu_gmres.py tests/test_gpu_small_cycle.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; fatal $rc tests
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh 3 "HH_SL_RES=0" "HH_SL_RES=1" -- python bench.py --no-cpu-baseline --const-steps 0 > $O/ab_slres.log 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/ab_slres.log; fatal $rc ab
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_bench -o run --output-format csv -- python3 bench.py --no-cpu-baseline --const-steps 0 > $O/rocprof_bench.log 2>&1; rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
python3 tools/cycle_timeline.py $O/rocprof_bench/run_kernel_trace.csv > $O/cycle_timeline.txt; tail -12 $O/cycle_timeline.txt
bash tools/_r05q.sh
