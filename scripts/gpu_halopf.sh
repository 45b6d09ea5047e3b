# Prefetching halo tiles 22-25: kernel tests, re-tune fprop/dgrad (x3, bf16), benches.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "halo" > gpurun_out/halopf_tests.log 2>&1 || { tail -30 gpurun_out/halopf_tests.log; exit 1; }
tail -1 gpurun_out/halopf_tests.log
timeout -k 10 100 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_pf_before.log 2>&1
echo "x3 before $(grep -o '"value": [0-9.]*' gpurun_out/bench_pf_before.log)"
timeout -k 10 400 python tools/tune_convs.py --impls x3,bf16 --only "fprop|,dgrad|" > gpurun_out/tunepf.log 2>&1
grep "sum_best" gpurun_out/tunepf.log
cp distributed_pytorch_amd/tuning/mi355x.json gpurun_out/mi355x.json
for impl in x3 bf16 x3; do
  timeout -k 10 150 python bench.py --steps 50 --warmup 10 --impl $impl > gpurun_out/benchpf_$impl.log 2>&1
  echo "$impl after $(grep -o '"value": [0-9.]*' gpurun_out/benchpf_$impl.log)"
done
