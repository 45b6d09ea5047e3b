# ResNet downsample branch: its BN applied inside the block's add + ReLU (no stored BN output)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_layers_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4rbn_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/r4rbn_tests.log; [ $rc -eq 0 ] || exit 1
BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=3 AB_ENVS="DPA_FUSE_RES_BN=0|DPA_FUSE_RES_BN=1" bash scripts/gpu_ab.sh || exit 1
