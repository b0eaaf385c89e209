# rocprofv3 kernel traces of the GMRES loop at BASELINE configs 1 and 2 (launch-bound sizes)
set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/t1
for c in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/t1/c$c -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/t1/c$c.log 2>&1 || exit $?
done
