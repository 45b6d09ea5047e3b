# ResNet-50 (bench_resnet.py) kernel trace + stats, and a plain timed run.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python bench_resnet.py --steps 20 --warmup 5 ${ARGS:-} > gpurun_out/rn_bench.log 2>&1 || { tail -20 gpurun_out/rn_bench.log; exit 1; }
tail -1 gpurun_out/rn_bench.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rn_trace -o run -- python3 $R/bench_resnet.py --steps 6 --warmup 3 ${ARGS:-} > $R/gpurun_out/rn_trace.log 2>&1 || { tail -20 $R/gpurun_out/rn_trace.log; exit 1; }
echo trace-ok
