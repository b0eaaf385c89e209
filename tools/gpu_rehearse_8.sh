# Rehearses the driver's 8-GPU bench (bench.py --gpus 8) on ONE GPU: 8 ranks under
# torch.distributed.run, all on device 0 -- the rendezvous, the watchdog bounds, the one-pass
# path across 8 slabs and the breakdown's allreduces per iteration at 8 processes.  Transport:
# RCCL over loopback (one NCCL_HOSTID per rank) if it accepts 8 ranks on one device, else the
# host-staged SHM transport; the line's `parallelism` names the one used.  ARGS are passed to
# bench.py (e.g. --grid 4096 --same-n 2048 for a reduced grid).  Rates are one card shared by 8
# processes, not scaling.  TRANSPORTS limits the transports tried (default "rccl shm").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/rehearse8}; mkdir -p $OUT
TAG=${TAG:-n8}
for tr in ${TRANSPORTS:-rccl shm}; do
  extra=""; [ $tr = rccl ] && extra="HH_RCCL_HOSTID_PER_RANK=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1"
  env HH_TRANSPORT=$tr HH_FORCE_DEVICE=0 $extra timeout -k 10 ${SECS:-600} python bench.py --gpus 8 "$@" \
    > $OUT/bench_${TAG}_$tr.log 2>&1
  rc=$?
  echo "transport $tr rc=$rc"
  if [ $rc -eq 0 ]; then
    grep '^{' $OUT/bench_${TAG}_$tr.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); g=d.get('gmres') or {}; s=d.get('same_n') or {}; print('N', d['n_gpus'], 'n', d['config']['n'], d['config']['parallelism'], 'value', d['value'], 'gmres', g.get('iters_per_s'), g.get('solve_path'), g.get('final_rel_presid'), 'same_n', json.dumps(s.get('breakdown', {}).get('gmres_per_iteration')))"
    exit 0
  fi
  tail -20 $OUT/bench_${TAG}_$tr.log
  case $rc in 124|137|134|139) exit $rc;; esac
  # a device fault reported as an error (HH_CHECK_HALO attributes it): nothing more on the GPU
  grep -q "illegal memory access\|FAULT at" $OUT/bench_${TAG}_$tr.log && exit 5
done
exit 1
