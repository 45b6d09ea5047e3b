# ResNet-50 weight gradients on a side stream: tests, A/B on bench_resnet, step trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_layers_gpu.py tests/test_bn_wide_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_ws_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4_ws_tests.log; [ $rc -eq 0 ] || exit 1
BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=3 AB_ENVS="DPA_WGRAD_STREAM=0|DPA_WGRAD_STREAM=1" bash scripts/gpu_ab.sh || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p_rn_ws -o rn -- python bench_resnet.py --steps 10 --warmup 5 > gpurun_out/r4p_rn_ws.log 2>&1; echo "prof rc=$?"
