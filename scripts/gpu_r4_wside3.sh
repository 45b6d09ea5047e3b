# side-stream wgrad: batched forks A/B (graph replay), plus the layer tests
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_ws3_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4_ws3_tests.log; [ $rc -eq 0 ] || exit 1
BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=3 AB_ENVS="DPA_WGRAD_STREAM=0|DPA_WGRAD_STREAM=1|DPA_WGRAD_BATCH=3|DPA_WGRAD_BATCH=8" bash scripts/gpu_ab.sh || exit 1
