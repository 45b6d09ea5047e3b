# forward finalize (column-major epilogue partials): 8 loads in flight per thread; tests + ResNet trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bn_gpu.py tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4fcm_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4fcm_tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/gpu_r4_rnprof.sh || exit 1
timeout -k 10 300 python bench_resnet.py --steps 40 --warmup 10 > gpurun_out/r4fcm_rn.json 2>&1; tail -1 gpurun_out/r4fcm_rn.json | cut -c1-150
