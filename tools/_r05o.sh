set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05o; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_spmv.py tests/test_gpu_variants.py tests/test_gpu_configs.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; fatal $rc tests
[ $rc -ne 0 ] && exit $rc
for g in 5792 11584 4096; do for med in marmousi const; do
bash tools/ab_env.sh 2 "HH_TILE_XCD=0" "HH_TILE_XCD=1" -- python bench.py --grid $g --medium $med --no-gmres --no-cpu-baseline --same-n 0 --const-steps 0 > $O/ab_xcd_${g}_$med.log 2>&1; rc=$?; echo "ab $g $med rc=$rc"; cat $O/ab_xcd_${g}_$med.log; fatal $rc ab
done; done
OUT=$O KNOBS=HH_TILE_XCD=1 timeout -k 10 600 bash tools/pmc_shapes.sh 5792:2 11584:8 > $O/pmc_shapes_xcd.log 2>&1; rc=$?; echo "shapes rc=$rc"; grep "tile_kernel" $O/pmc_shapes_xcd.log; fatal $rc shapes
