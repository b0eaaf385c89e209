set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05p; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
for N in 2 4; do
HH_TRANSPORT=rccl HH_FORCE_DEVICE=0 HH_RCCL_HOSTID_PER_RANK=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 timeout -k 10 400 python bench.py --gpus $N --no-cpu-baseline --const-steps 0 --same-n 0 > $O/rccl_n$N.log 2>&1; rc=$?; echo "rccl N=$N rc=$rc"; grep '^{' $O/rccl_n$N.log | cut -c1-300; grep -i "error\|illegal" $O/rccl_n$N.log | head -5
[ $rc -ne 0 ] && exit $rc
done
