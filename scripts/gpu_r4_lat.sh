# latency-bound critical-path kernels: fc_ce row kernel (W loads batched), BN finalize (16 partial
# rows per thread in flight); tests, then the step kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_bn_gpu.py tests/test_fused_gpu.py tests/test_layer0_gpu.py tests/test_parity256_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4lat_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4lat_tests.log; [ $rc -eq 0 ] || exit 1
TAG=r4lat bash scripts/gpu_profile.sh || exit 1
timeout -k 10 200 python bench.py --gpus 1 --steps 100 --warmup 20 > gpurun_out/r4lat_bench.json 2> gpurun_out/r4lat_bench.err; echo "bench rc=$?"; tail -1 gpurun_out/r4lat_bench.json | cut -c1-160
