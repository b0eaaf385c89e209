set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05rb; mkdir -p $O
summ() { grep '^{' $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d.get('gmres') or {}; print('N', d['n_gpus'], 'n', d['config']['n'], d['config']['parallelism'], 'value', d['value'], 'gmres', g.get('iters_per_s'), g.get('solve_path'), g.get('final_rel_presid'))"; }
HH_TRANSPORT=shm HH_FORCE_DEVICE=0 timeout -k 10 600 python bench.py --gpus 8 --no-cpu-baseline --same-n 0 > $O/rehearse8_default_shm.log 2>&1; rc=$?; echo "shm8 rc=$rc"; [ $rc -eq 0 ] && summ $O/rehearse8_default_shm.log
case $rc in 0) ;; *) exit $rc;; esac
# the default weak grid over RCCL loopback once more on the final tree (faulted once in r05f)
HH_TRANSPORT=rccl HH_FORCE_DEVICE=0 HH_RCCL_HOSTID_PER_RANK=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 timeout -k 10 600 python bench.py --gpus 8 --no-cpu-baseline --same-n 0 > $O/rehearse8_default_rccl.log 2>&1; rc=$?; echo "rccl8 rc=$rc"; [ $rc -eq 0 ] && summ $O/rehearse8_default_rccl.log; grep -i "fault\|illegal\|hh_err" $O/rehearse8_default_rccl.log | sort | uniq -c | head -5
exit 0
