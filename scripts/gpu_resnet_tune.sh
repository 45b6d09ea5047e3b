# ResNet-50: kernel/layer tests, conv autotune of the table's missing entries
# (copied to gpurun_out/), then same-box A/Bs of the BN dy pass and of HIP-graph replay.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_bn_gpu.py tests/test_layers_gpu.py tests/test_ops_gpu.py -k "${TESTS_K:-dgrad or bn or layers or resnet or ops}" \
  > gpurun_out/rn3_tests.log 2>&1 || { tail -40 gpurun_out/rn3_tests.log; exit 1; }
tail -1 gpurun_out/rn3_tests.log
timeout -k 10 600 python bench_resnet.py --autotune --steps 5 --warmup 2 > gpurun_out/rn_autotune.log 2>&1 || { tail -20 gpurun_out/rn_autotune.log; exit 1; }
cp distributed_pytorch_amd/tuning/generic_mi355x.json gpurun_out/generic_mi355x.json
AB_ENVS="${AB:-X=0|X=1}" REPS=3 BENCH=bench_resnet.py STEPS=100 WARMUP=10 bash scripts/gpu_ab.sh
REPS=2 BENCH=bench_resnet.py STEPS=100 WARMUP=10 ARGS="--graph on" bash scripts/gpu_ab.sh
