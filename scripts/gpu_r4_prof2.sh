export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp
DPA_FORCE_COMM=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/r4p_rccl1b -o run -- python3 $R/bench.py --steps 30 --warmup 5 > $R/gpurun_out/r4p_rccl1b.log 2>&1 && echo "rccl1 trace ok"
