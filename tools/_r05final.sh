set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05final; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
# the driver's exact command under rocprofv3 (kernel trace + stats), for the roofline evidence
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/rocprof_driver -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_rocprof.log 2>&1; rc=$?; echo "rocprof driver rc=$rc"; grep '^{' $O/driver_rocprof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'gmres', d['gmres']['iters_per_s'])"; fatal $rc rocprof
grep "tile_kernel<0, false, 4" $O/rocprof_driver/run_kernel_stats.csv | cut -c1-200
