set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05m; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
bash tools/ab_env.sh 2 "HH_FUSED_ROWS=8" "HH_FUSED_ROWS=16" "HH_FUSED_ROWS=32" -- python bench.py --config 2 --no-cpu-baseline > $O/ab_rows_c2.log 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/ab_rows_c2.log; fatal $rc ab
timeout -k 10 300 python tools/tune_stencil.py --n 4096 --variants 98,99,100,101,102,104,132,164 --rpbs 16 --grids 0 --medium const --rotate 3 --rounds 3 > $O/tune_tiles_const.log 2>&1; rc=$?; echo "tune rc=$rc"; tail -10 $O/tune_tiles_const.log; fatal $rc tune
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_bench -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/rocprof_bench.log 2>&1; rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
python3 - <<'PY' | tee $O/tile_durations.txt
import csv, statistics as st
rows = list(csv.DictReader(open("gpurun_out/r05m/rocprof_bench/run_kernel_trace.csv")))
for key in ("tile_kernel<0, true, 4", "tile_kernel<0, false, 4"):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if key in r["Kernel_Name"]]
    if d:
        print(f"{key}: {len(d)} launches, avg {st.mean(d):.1f} median {st.median(d):.1f} min {min(d):.1f} us; last 200: avg {st.mean(d[-200:]):.1f} median {st.median(d[-200:]):.1f}")
PY
for ctr in FETCH_SIZE WRITE_SIZE; do
  HH_FUSED_ROWS=16 PRECOND=jacobi MODES=fused timeout -s KILL 300 rocprofv3 --pmc $ctr -d $O/pmc_1024r16_$ctr -o run --output-format csv -- python3 tools/ab_krylov_mode.py 1024 64 1 > $O/pmc_1024r16_$ctr.log 2>&1; rc=$?; echo "pmc $ctr rc=$rc"; fatal $rc pmc
done
python3 tools/pmc_fused.py $O/pmc_1024r16_FETCH_SIZE/run_counter_collection.csv $O/pmc_1024r16_WRITE_SIZE/run_counter_collection.csv --n 1024 --medium const --precond jacobi --restart 20 --knobs HH_FUSED_ROWS=16 --merge $O/r05_pmc_fused.json | tee $O/pmc_1024r16.txt
timeout -k 10 400 python3 tools/bench_sweep.py --maxiter 0 1023 4095 > $O/sweep_mem.log 2>&1; rc=$?; echo "sweep rc=$rc"; tail -3 $O/sweep_mem.log; fatal $rc sweep
