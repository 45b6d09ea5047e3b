# ResNet-50 generic path: layer tests, op breakdown, bench (bf16, batch 128).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rn_tests.log 2>&1 || { tail -40 gpurun_out/rn_tests.log; exit 1; }
tail -1 gpurun_out/rn_tests.log
timeout -k 10 200 python bench_resnet.py --batch 128 > gpurun_out/bench_resnet.log 2>&1
echo "resnet $(grep -o '"value": [0-9.]*' gpurun_out/bench_resnet.log)"
timeout -k 10 200 python tools/resnet_ops.py > gpurun_out/rn_ops.log 2>&1
echo ops-ok
