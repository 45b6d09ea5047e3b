# Round-2 checks: new RCCL / batch-256 parity tests, the whole GPU suite, bench (null comm and
# 1-rank RCCL with the diagnostic phase).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py tests/test_parity256_gpu.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r2a_new_tests.log 2>&1 || { tail -60 gpurun_out/r2a_new_tests.log; exit 1; }
tail -3 gpurun_out/r2a_new_tests.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2a_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r2a_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r2a_gpu_tests.log
timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/r2a_bench.log 2>&1 || { tail -20 gpurun_out/r2a_bench.log; exit 1; }
tail -1 gpurun_out/r2a_bench.log
DPA_FORCE_COMM=1 timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/r2a_bench_rccl1.log 2>&1 || { tail -20 gpurun_out/r2a_bench_rccl1.log; exit 1; }
tail -1 gpurun_out/r2a_bench_rccl1.log
