# Rehearses the driver's multi-GPU bench at its default (weak-scaling) sizes on ONE GPU: N ranks
# under torch.distributed.run, all on device 0, halo/allreduce through the host-staged SHM
# transport (RCCL refuses two ranks on one device).  Checks orchestration and memory at the
# real grid sizes (n = 5792 at N = 2, 8192 at N = 4), then the BASELINE strong-scaling presets
# (config 4: 8192^2 on 2 ranks, config 5: 16384^2 on 4); the throughput is NOT a scaling number.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; OUT=gpurun_out/rehearse; mkdir -p $OUT
for N in 2 4; do
  HH_TRANSPORT=shm HH_FORCE_DEVICE=0 timeout -k 10 400 python bench.py --gpus $N > $OUT/bench_n$N.log 2>&1 || { tail -30 $OUT/bench_n$N.log; exit 1; }
  grep '^{' $OUT/bench_n$N.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N', d['n_gpus'], 'n', d['config']['n'], 'value', d['value'], 'gmres', d['gmres']['iters_per_s'], d['gmres']['final_rel_presid'])"
done
for cfg in "4 2" "5 4"; do
  set -- $cfg
  HH_TRANSPORT=shm HH_FORCE_DEVICE=0 timeout -k 10 500 python bench.py --config $1 --gpus $2 > $OUT/bench_c$1_n$2.log 2>&1 || { tail -30 $OUT/bench_c$1_n$2.log; exit 1; }
  grep '^{' $OUT/bench_c$1_n$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('config', $1, 'N', d['n_gpus'], 'n', d['config']['n'], d['scaling'], 'value', d['value'], 'gmres', d['gmres']['iters_per_s'], d['gmres']['final_rel_presid'])"
done
