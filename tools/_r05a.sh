set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_krylov_modes.py -k "keep_kernel or fused_pass_matches_lagged or fused_pass_matches_reference or keep_knob" > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh 2 "HH_SLK=0" "HH_SLK=1" -- python bench.py --no-cpu-baseline > $O/ab.log 2>&1; echo "ab rc=$?"; cat $O/ab.log
