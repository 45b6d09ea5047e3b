# BN backward reduce with 256-thread blocks: BN/engine/layer tests, x3/bf16 benches, ResNet, trace.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_layers_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bnbwd_tests.log 2>&1 || { tail -30 gpurun_out/bnbwd_tests.log; exit 1; }
tail -1 gpurun_out/bnbwd_tests.log
for impl in x3 bf16; do
  timeout -k 10 150 python bench.py --steps 50 --warmup 10 --impl $impl > gpurun_out/bench_bnb_$impl.log 2>&1
  echo "$impl $(grep -o '"value": [0-9.]*' gpurun_out/bench_bnb_$impl.log)"
done
timeout -k 10 200 python bench_resnet.py --batch 128 > gpurun_out/bench_resnet.log 2>&1
echo "resnet $(grep -o '"value": [0-9.]*' gpurun_out/bench_resnet.log)"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof.log 2>&1
echo prof-ok
