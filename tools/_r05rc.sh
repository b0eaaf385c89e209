set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05rc; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_configs.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; fatal $rc tests
[ $rc -ne 0 ] && exit $rc
summ() { grep '^{' $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d.get('gmres') or {}; print('N', d['n_gpus'], 'n', d['config']['n'], d['config']['parallelism'], 'value', d['value'], 'gmres', g.get('iters_per_s'), g.get('solve_path'), g.get('final_rel_presid'))"; }
HH_TRANSPORT=rccl HH_FORCE_DEVICE=0 HH_RCCL_HOSTID_PER_RANK=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 timeout -k 10 600 python bench.py --gpus 8 --no-cpu-baseline --same-n 0 > $O/rehearse8_default_rccl.log 2>&1; rc=$?; echo "rccl8 rc=$rc"; [ $rc -eq 0 ] && summ $O/rehearse8_default_rccl.log; grep -i "illegal\|hh_err" $O/rehearse8_default_rccl.log | sort | uniq -c | head -3
exit 0
