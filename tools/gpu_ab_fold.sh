# Bitwise A/B of the GMRES fold (one launch fewer per iteration) against the previous build
# (tmp_ab/libold.so, built from the previous commit with OUT=/root/repo/tmp_ab/libold.so), then the quick GPU check.
set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
HH_LIB_PATH=$PWD/tmp_ab/libold.so timeout -k 10 120 python tools/ab_gmres_bits.py dump gpurun_out/ab/old.npz || exit $?
timeout -k 10 120 python tools/ab_gmres_bits.py dump gpurun_out/ab/new.npz || exit $?
python tools/ab_gmres_bits.py compare gpurun_out/ab/old.npz gpurun_out/ab/new.npz
bash tools/gpu_quick.sh q2
