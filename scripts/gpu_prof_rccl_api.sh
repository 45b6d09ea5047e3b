# Kernel + HIP API trace of the 1-rank RCCL step: host enqueue time vs GPU time per kernel.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && DPA_FORCE_COMM=1 timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/gpurun_out/prof_rccl_api -o run -- python $R/bench.py --steps 10 --warmup 5 --diag-steps 0 > $R/gpurun_out/prof_rccl_api.log 2>&1 || { tail -20 $R/gpurun_out/prof_rccl_api.log; exit 1; }
tail -1 $R/gpurun_out/prof_rccl_api.log
