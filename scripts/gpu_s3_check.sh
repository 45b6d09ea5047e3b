# Targeted GPU tests of the sync/comm paths + default benches (null comm and 1-rank RCCL).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py tests/test_rccl_gpu.py tests/test_ops_gpu.py tests/test_signal_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/s3c_tests.log 2>&1 || { tail -40 gpurun_out/s3c_tests.log; exit 1; }
tail -1 gpurun_out/s3c_tests.log
timeout -k 10 150 python bench.py --steps 100 --warmup 20 > gpurun_out/s3c_bench.log 2>&1 || { tail -20 gpurun_out/s3c_bench.log; exit 1; }
tail -1 gpurun_out/s3c_bench.log
DPA_FORCE_COMM=1 timeout -k 10 150 python bench.py --steps 100 --warmup 20 > gpurun_out/s3c_bench_rccl1.log 2>&1 || { tail -20 gpurun_out/s3c_bench_rccl1.log; exit 1; }
tail -1 gpurun_out/s3c_bench_rccl1.log
