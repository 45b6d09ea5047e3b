export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py -x -q --timeout 120 --timeout-method thread -k "two_ranks or agree or ipc" > gpurun_out/r4_t4.log 2>&1; echo "multirank rc=$?"; tail -4 gpurun_out/r4_t4.log
cd /tmp
DPA_FORCE_COMM=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4p_rccl1 -o run -- python3 $R/bench.py --steps 30 --warmup 5 > $R/gpurun_out/r4p_rccl1.log 2>&1 && echo "rccl1 trace ok" && tail -1 $R/gpurun_out/r4p_rccl1.log | cut -c1-160
cd $R
timeout -k 10 100 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_drv2.log 2>&1 && tail -1 gpurun_out/r4_drv2.log | cut -c1-160
