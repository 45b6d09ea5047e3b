# 3x3/s2 max-pool backward specialisation (2x2 input pixels per thread)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4pb_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4pb_tests.log; [ $rc -eq 0 ] || exit 1
BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=3 AB_ENVS="DPA_POOL_K3S2=0|DPA_POOL_K3S2=1" bash scripts/gpu_ab.sh || exit 1
