# Round validation on one MI355X: full GPU test suite, x3/bf16/fp32 benches, ResNet-50 bench,
# and a kernel-trace profile of the headline bench. Every GPU step has its own time limit and
# the script stops at the first failure.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for impl in x3 bf16 fp32; do
  timeout -k 10 150 python bench.py --steps 50 --warmup 10 --impl $impl > gpurun_out/bench_$impl.log 2>&1
  echo "$impl $(grep -o '"value": [0-9.]*' gpurun_out/bench_$impl.log)"
done
timeout -k 10 200 python bench_resnet.py --batch 128 > gpurun_out/bench_resnet.log 2>&1
echo "resnet $(grep -o '"value": [0-9.]*' gpurun_out/bench_resnet.log)"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof.log 2>&1
echo prof-ok
