set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05u; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
for R in 8 16; do
HH_FUSED_ROWS=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_r$R -o run --output-format csv -- python3 bench.py --config 2 --no-cpu-baseline > $O/rocprof_r$R.log 2>&1; rc=$?; echo "rocprof R=$R rc=$rc"; fatal $rc rocprof
python3 tools/fused_tbps.py $O/rocprof_r$R/run_kernel_stats.csv 1024 8 > $O/tbps_r$R.txt 2>&1
done
paste $O/tbps_r8.txt $O/tbps_r16.txt | cut -c1-160
