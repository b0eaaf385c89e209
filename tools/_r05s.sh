set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05s; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
# tile shapes with non-temporal u loads (halo rows re-read from HBM / MALL instead of L2) vs cached
for med in marmousi const; do for n in 4096 8192; do
timeout -k 10 400 python tools/tune_stencil.py --n $n --variants 100,104,102,116,118,120 --rpbs 16 --grids 0 --medium $med --rotate 3 --rounds 3 > $O/tune_ntu_${med}_$n.log 2>&1; rc=$?; echo "tune $med $n rc=$rc"; tail -7 $O/tune_ntu_${med}_$n.log; fatal $rc tune
done; done
