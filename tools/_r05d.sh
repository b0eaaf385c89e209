set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05d; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
C=SQ_WAVES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_WAIT_INST_LDS
for v in old d1 d2; do
  case $v in old) E="HH_SLK=0";; d1) E="HH_SLK=1 HH_LIB_PATH=abl/libhh_slk_d1.so HH_LIB_AB=1";; d2) E="HH_SLK=1";; esac
  env $E PRECOND=sl MODES=fused timeout -s KILL 240 rocprofv3 --pmc $C -d $O/sq_$v -o run --output-format csv -- python3 tools/ab_krylov_mode.py 4096 100 1 > $O/sq_$v.log 2>&1; rc=$?; echo "$v rc=$rc"; fatal $rc sq_$v
  python3 tools/pmc_sq.py $O/sq_$v/run_counter_collection.csv --match "fused_sl" | tee $O/sq_$v.txt
done
