# deferred optimizer step: tests + VGG A/B (interleaved, steady 100/20) + driver-style runs
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_defer_gpu.py tests/test_ops_gpu.py tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_defer_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4_defer_tests.log; [ $rc -eq 0 ] || exit 1
REPS=3 AB_ENVS="DPA_DEFER_UPDATE=0|DPA_DEFER_UPDATE=1" bash scripts/gpu_ab.sh || exit 1
STEPS=20 WARMUP=5 REPS=2 AB_ENVS="DPA_DEFER_UPDATE=0|DPA_DEFER_UPDATE=1" bash scripts/gpu_ab.sh || exit 1
