set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05e; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_krylov_modes.py -k "keep_kernel or alternating or fused_pass_matches_reference or fused_pass_matches_lagged or virtual_slabs or lds_kept" > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; fatal $rc tests
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh 2 "HH_SLK=0" "HH_SLK=1" "HH_SLK=7" -- python bench.py --no-cpu-baseline --const-steps 0 > $O/ab_slk.log 2>&1; rc=$?; echo "ab_slk rc=$rc"; cat $O/ab_slk.log; fatal $rc ab_slk
for v in 0 1; do
HH_SLK=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_slk$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --const-steps 0 > $O/rocprof_slk$v.log 2>&1; rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
python3 tools/fused_tbps.py $O/rocprof_slk$v/run_kernel_stats.csv 4096 8 | tee $O/slk${v}_tbps.txt
done
C=SQ_WAVES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_WAIT_INST_LDS
HH_SLK=1 PRECOND=sl MODES=fused timeout -s KILL 240 rocprofv3 --pmc $C -d $O/sq_slk -o run --output-format csv -- python3 tools/ab_krylov_mode.py 4096 100 1 > $O/sq_slk.log 2>&1; rc=$?; echo "sq rc=$rc"; fatal $rc sq
python3 tools/pmc_sq.py $O/sq_slk/run_counter_collection.csv --match "fused_sl" | tee $O/sq_slk.txt
