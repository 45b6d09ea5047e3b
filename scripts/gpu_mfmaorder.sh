# Product-major MFMA order: kernel tests, conv sums (tune with --only fprop/dgrad), benches.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mo_tests.log 2>&1 || { tail -30 gpurun_out/mo_tests.log; exit 1; }
tail -1 gpurun_out/mo_tests.log
timeout -k 10 500 python tools/tune_convs.py --impls x3,bf16 > gpurun_out/tune_mo.log 2>&1
grep "sum_best" gpurun_out/tune_mo.log
cp distributed_pytorch_amd/tuning/mi355x.json gpurun_out/mi355x.json
for impl in x3 bf16 x3; do
  timeout -k 10 150 python bench.py --steps 50 --warmup 10 --impl $impl > gpurun_out/bench_mo_$impl.log 2>&1
  echo "$impl $(grep -o '"value": [0-9.]*' gpurun_out/bench_mo_$impl.log)"
done
