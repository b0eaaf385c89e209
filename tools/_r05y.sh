set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05y; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
# run-to-run spread on one box, the final tree: 5 runs each of config 2 and the default (config 3) line
bash tools/ab_env.sh 5 "HH_NOTHING=0" -- python bench.py --config 2 --no-cpu-baseline > $O/spread_c2.log 2>&1; rc=$?; echo "c2 rc=$rc"; cat $O/spread_c2.log; fatal $rc c2
bash tools/ab_env.sh 5 "HH_NOTHING=0" -- python bench.py --no-cpu-baseline --const-steps 0 > $O/spread_c3.log 2>&1; rc=$?; echo "c3 rc=$rc"; cat $O/spread_c3.log; fatal $rc c3
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.log 2>&1; rc=$?; echo "driver rc=$rc"; grep '^{' $O/driver.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['gmres']; print('value', d['value'], 'gmres', g['iters_per_s'], g['solve_path'])"; fatal $rc driver
