set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05n; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
OUT=$O timeout -k 10 1000 bash tools/pmc_shapes.sh > $O/pmc_shapes.log 2>&1; rc=$?; echo "shapes rc=$rc"; tail -30 $O/pmc_shapes.log; fatal $rc shapes
