set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05b; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_krylov_modes.py -k "keep_kernel or fused_pass_matches_lagged or fused_pass_matches_reference or keep_knob or alternating" > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 $O/tests.log; fatal $rc tests
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh 2 "HH_SLK=0" "HH_SLK=1" -- python bench.py --no-cpu-baseline --const-steps 0 > $O/ab_slk.log 2>&1; rc=$?; echo "ab_slk rc=$rc"; cat $O/ab_slk.log; fatal $rc ab_slk
bash tools/ab_env.sh 2 "HH_FUSED_ALT=0" "HH_FUSED_ALT=1" -- python bench.py --config 2 --no-cpu-baseline > $O/ab_alt.log 2>&1; rc=$?; echo "ab_alt rc=$rc"; cat $O/ab_alt.log; fatal $rc ab_alt
HH_SLK=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_slk -o run --output-format csv -- python3 bench.py --no-cpu-baseline --const-steps 0 > $O/rocprof_slk.log 2>&1; rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
python3 tools/fused_tbps.py $O/rocprof_slk/run_kernel_stats.csv 4096 8 | tee $O/slk_tbps.txt
timeout -k 10 300 python tools/tune_stencil.py --n 4096 --variants 100,162,164,166,168 --rpbs 16 --grids 0 --medium const --rotate 3 --rounds 3 > $O/tune_persist_const.log 2>&1; rc=$?; echo "tune rc=$rc"; tail -8 $O/tune_persist_const.log; fatal $rc tune
