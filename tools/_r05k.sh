set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05k; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_krylov_modes.py -k "lag_reduce or cycle_end_merge or matches_lagged or keep_kernel" > $O/tests_k.log 2>&1; rc=$?; echo "tests_k rc=$rc"; tail -3 $O/tests_k.log; fatal $rc tests_k
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh 3 "HH_LAG_RED=0" "HH_LAG_RED=1" -- python bench.py --config 2 --no-cpu-baseline > $O/ab_lagred.log 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/ab_lagred.log; fatal $rc ab
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_c2 -o run --output-format csv -- python3 bench.py --config 2 --no-cpu-baseline > $O/rocprof_c2.log 2>&1; rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
grep -E "cycle_coef|lag_red|gmres_lag|reduce_kernel|gmres_solve|cycle_end|cycle_finish" $O/rocprof_c2/run_kernel_stats.csv | cut -c1-200
echo "--- RCCL loopback probe, 8 ranks on one GPU (no kernel of this package)"
HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 tools/rccl_loopback_probe.py 4096 11584 > $O/rccl_probe.log 2>&1; rc=$?; echo "probe rc=$rc"; grep -E "^n=|Error|error" $O/rccl_probe.log | head -20; fatal $rc probe
