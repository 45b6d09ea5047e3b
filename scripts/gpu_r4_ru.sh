# wide BN backward reduce: four rows in flight per thread (DPA_BN_WIDE_RU=4) vs two, ResNet-50 bf16
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bn_wide_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4ru_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4ru_tests.log; [ $rc -eq 0 ] || exit 1
BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=3 AB_ENVS="DPA_BN_WIDE_RU=2|DPA_BN_WIDE_RU=4" bash scripts/gpu_ab.sh || exit 1
