set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05f; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_dist.py -k "fused_pass_ranks" > $O/tests_dist.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 $O/tests_dist.log; fatal $rc tests
[ $rc -ne 0 ] && exit $rc
OUT=$O TAG=reduced SECS=500 bash tools/gpu_rehearse_8.sh --grid 4096 --same-n 2048 --steps 50 --warmup 20 --gmres-iters 20 --const-steps 50 --same-n-steps 50; rc=$?; echo "rehearse reduced rc=$rc"; fatal $rc rehearse
OUT=$O TAG=default SECS=700 bash tools/gpu_rehearse_8.sh --steps 20 --warmup 5; rc=$?; echo "rehearse default rc=$rc"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_c2 -o run --output-format csv -- python3 bench.py --config 2 --no-cpu-baseline > $O/rocprof_c2.log 2>&1; echo "rocprof c2 rc=$?"
