# 1-rank RCCL kernel trace (check the last bucket's update is ordered after every producer) and the
# per-kernel PMC passes of the x3 step (single stream so counters are not mixed).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp
DPA_FORCE_COMM=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rccl -o run -- python3 $R/bench.py --steps 20 --warmup 5 --diag-steps 0 > $R/gpurun_out/prof_rccl.log 2>&1
tail -1 $R/gpurun_out/prof_rccl.log
bash $R/scripts/pmc_conv.sh
