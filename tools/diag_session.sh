set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in "3 2 6" "3 1 6" "4 1 4" "2 2 4"; do
  timeout -k 10 300 python -u tools/stress_dist.py multi $cfg > gpurun_out/diag_multi.log 2>&1; rc=$?
  echo "cfg $cfg rc=$rc"; grep -E "gmres none|apply" gpurun_out/diag_multi.log | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit $rc
done
