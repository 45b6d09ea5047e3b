# Host enqueue time and Python profile of the bench step (null comm and 1-rank RCCL).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python tools/host_profile.py --comm null > gpurun_out/host_null.log 2>&1 || { tail -20 gpurun_out/host_null.log; exit 1; }
head -1 gpurun_out/host_null.log
MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 timeout -k 10 200 python tools/host_profile.py --comm rccl > gpurun_out/host_rccl.log 2>&1 || { tail -20 gpurun_out/host_rccl.log; exit 1; }
head -1 gpurun_out/host_rccl.log
