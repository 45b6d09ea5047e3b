# 32-bit index max-pool kernels: tests, ResNet bench, kernel times
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py -x -q -k "maxpool" --timeout 200 --timeout-method thread > gpurun_out/r4_pool_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4_pool_tests.log; [ $rc -eq 0 ] || exit 1
BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=2 AB_ENVS="X=0" bash scripts/gpu_ab.sh || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p_rn_pool -o rn -- python bench_resnet.py --steps 10 --warmup 5 > gpurun_out/r4p_rn_pool.log 2>&1; echo "prof rc=$?"
