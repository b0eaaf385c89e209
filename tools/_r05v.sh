set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05v; mkdir -p $O
summ() { grep '^{' $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d.get('gmres') or {}; s=d.get('same_n') or {}; b=d.get('breakdown') or {}; print('N', d['n_gpus'], 'n', d['config']['n'], d['config']['parallelism'], 'value', d['value'], 'gmres', g.get('iters_per_s'), g.get('solve_path'), 'traffic', d['roofline'].get('traffic_vs_algorithmic'), g.get('pass_traffic_vs_algorithmic'), 'allreduces/it', (s.get('breakdown') or {}).get('gmres_per_iteration', {}).get('allreduces'))"; }
HH_TRANSPORT=rccl HH_FORCE_DEVICE=0 HH_RCCL_HOSTID_PER_RANK=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 timeout -k 10 600 python bench.py --gpus 8 --grid 4096 --same-n 4096 --no-cpu-baseline > $O/rehearse8_reduced_rccl.log 2>&1; rc=$?; echo "rccl reduced rc=$rc"; [ $rc -eq 0 ] && summ $O/rehearse8_reduced_rccl.log
case $rc in 124|137|134|139) exit $rc;; esac
HH_TRANSPORT=shm HH_FORCE_DEVICE=0 timeout -k 10 600 python bench.py --gpus 8 --no-cpu-baseline > $O/rehearse8_default_shm.log 2>&1; rc=$?; echo "shm default rc=$rc"; [ $rc -eq 0 ] && summ $O/rehearse8_default_shm.log
exit 0
