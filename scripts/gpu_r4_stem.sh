# ResNet stem: BN + ReLU applied inside the max-pool's loads (no BN output tensor)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_layers_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4stem_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4stem_tests.log; [ $rc -eq 0 ] || exit 1
BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=3 AB_ENVS="DPA_FUSE_BN_POOL=0|DPA_FUSE_BN_POOL=1" bash scripts/gpu_ab.sh || exit 1
