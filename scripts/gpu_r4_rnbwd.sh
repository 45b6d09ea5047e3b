# ResNet-50: bf16 BN backward reduce always in the 1024-thread geometry (new default) vs forced
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bn_wide_gpu.py tests/test_layers_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_rnbwd_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4_rnbwd_tests.log; [ $rc -eq 0 ] || exit 1
BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=3 AB_ENVS="X=0|DPA_BN_BWD_BLOCK=1024" bash scripts/gpu_ab.sh || exit 1
