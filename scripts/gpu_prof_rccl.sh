# Kernel trace of the 1-rank RCCL step (DDP mode, fused per-bucket SGD on the comm stream).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && DPA_FORCE_COMM=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rccl -o run -- python $R/bench.py --steps 20 --warmup 5 --diag-steps 0 > $R/gpurun_out/prof_rccl.log 2>&1 || { tail -20 $R/gpurun_out/prof_rccl.log; exit 1; }
tail -1 $R/gpurun_out/prof_rccl.log
