set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05zz; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; fatal $rc tests
[ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; fatal $rc smoke
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.log 2>&1; rc=$?; echo "driver rc=$rc"; grep '^{' $O/driver.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['gmres']; print('value', d['value'], 'frac', d['roofline']['frac'], 'gmres', g['iters_per_s'], g['solve_path'], 'pass', g['pass_GBps'], 'const', d['spmv_constant_medium']['value'], 'cpu', d['cpu_baseline']['gmres_sample'][:60])"; fatal $rc driver
for c in 1 2 4 5; do
timeout -k 10 400 python3 bench.py --config $c --no-cpu-baseline > $O/config$c.log 2>&1; rc=$?; echo "config $c rc=$rc"; grep '^{' $O/config$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d.get('gmres') or {}; print('value', d['value'], 'gmres', g.get('iters_per_s'), g.get('solve_path'), 'pass', g.get('pass_GBps'), g.get('pass_traffic_vs_algorithmic'))"; fatal $rc config$c
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_bench -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/rocprof_bench.log 2>&1; rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
python3 tools/fused_tbps.py $O/rocprof_bench/run_kernel_stats.csv 4096 8 > $O/slk_tbps.txt 2>&1; tail -3 $O/slk_tbps.txt
