# bf16 16-byte-lane BN apply passes: bitwise tests, the one-launch BN tests, ResNet-50 A/B and profile
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_bn_wide_gpu.py tests/test_bn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_wide_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4_wide_tests.log; [ $rc -eq 0 ] || exit 1
BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=3 AB_ENVS="DPA_BN_WIDE=0|DPA_BN_WIDE=1 DPA_BN_WIDE_RED=0|DPA_BN_WIDE=1" bash scripts/gpu_ab.sh || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p_rn_wide -o rn -- python bench_resnet.py --steps 10 --warmup 5 > gpurun_out/r4p_rn_wide.log 2>&1; echo "prof rc=$?"
