# final-tree ResNet-50 kernel trace (bench_resnet.py, graph replay) for the per-kernel table
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rn4_trace -o run -- python3 $R/bench_resnet.py --steps 20 --warmup 5 > $R/gpurun_out/rn4_trace.log 2>&1 || { tail -20 $R/gpurun_out/rn4_trace.log; exit 1; }
echo trace-ok
