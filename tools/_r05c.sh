set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05c; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_krylov_modes.py -k "keep_kernel or alternating or fused_pass_matches_reference" > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; fatal $rc tests
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh 2 "HH_SLK=0" "HH_SLK=1" "HH_SLK=1 HH_LIB_PATH=abl/libhh_slk_d1.so HH_LIB_AB=1" -- python bench.py --no-cpu-baseline --const-steps 0 > $O/ab_slk.log 2>&1; rc=$?; echo "ab_slk rc=$rc"; cat $O/ab_slk.log; fatal $rc ab_slk
HH_SLK=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_slk -o run --output-format csv -- python3 bench.py --no-cpu-baseline --const-steps 0 > $O/rocprof_slk.log 2>&1; rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
python3 tools/fused_tbps.py $O/rocprof_slk/run_kernel_stats.csv 4096 8 | tee $O/slk_tbps.txt
