set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05t; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_spmv.py tests/test_gpu_variants.py tests/test_gpu_configs.py tests/test_gpu_krylov_modes.py -k "not lagged" > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; fatal $rc tests
[ $rc -ne 0 ] && exit $rc
for c in 4 5; do
timeout -k 10 400 python3 bench.py --config $c --no-cpu-baseline > $O/config$c.log 2>&1; rc=$?; echo "config $c rc=$rc"; grep '^{' $O/config$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d.get('gmres') or {}; print('value', d['value'], 'gmres', g.get('iters_per_s'), 'traffic', d['roofline'].get('traffic_vs_algorithmic'), d['roofline']['kernel'])"; fatal $rc config$c
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/driver.log 2>&1; rc=$?; echo "driver rc=$rc"; grep '^{' $O/driver.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'const', d['spmv_constant_medium'])"; fatal $rc driver
OUT=$O timeout -k 10 900 bash tools/pmc_shapes.sh > $O/pmc_shapes.log 2>&1; rc=$?; echo "shapes rc=$rc"; grep "const s5" $O/pmc_shapes.log; fatal $rc shapes
