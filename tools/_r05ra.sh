set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05ra; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; fatal $rc tests
[ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; fatal $rc smoke
HH_TRANSPORT=shm HH_FORCE_DEVICE=0 timeout -k 10 400 python bench.py --gpus 2 --no-cpu-baseline --const-steps 0 --same-n 0 > $O/rehearse2_shm.log 2>&1; rc=$?; echo "shm2 rc=$rc"; grep '^{' $O/rehearse2_shm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['gmres']; print('value', d['value'], 'gmres', g['iters_per_s'], g['solve_path'], g['final_rel_presid'])"; fatal $rc shm2
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.log 2>&1; rc=$?; echo "driver rc=$rc"; grep '^{' $O/driver.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['gmres']; print('value', d['value'], 'gmres', g['iters_per_s'], g['solve_path'])"; fatal $rc driver
