set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05w2; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
# band heights of the shifted-Laplace passes at 4096^2: HH_SLK_ROWS (K >= 2, one block per CU;
# default 256 = 16 bands x 16 strips = 256 tiles) and HH_FUSED_ROWS (the K = 1 two-block pass;
# default 32)
bash tools/ab_env.sh 2 "HH_SLK_ROWS=256" "HH_SLK_ROWS=128" "HH_SLK_ROWS=86" "HH_FUSED_ROWS=43" "HH_FUSED_ROWS=64" "HH_FUSED_ROWS=16" -- python bench.py --no-cpu-baseline --const-steps 0 > $O/ab_sl_rows.log 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/ab_sl_rows.log; fatal $rc ab
