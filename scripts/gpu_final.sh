# Round-end validation: full GPU suite, smoke(), benches (x3 twice, bf16, fp32), ResNet-50, 1-rank
# RCCL bench, kernel-trace profile of the headline bench.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for impl in x3 bf16 fp32 x3; do
  timeout -k 10 150 python bench.py --steps 50 --warmup 10 --impl $impl > gpurun_out/bench_$impl.log 2>&1
  echo "$impl $(grep -o '"value": [0-9.]*' gpurun_out/bench_$impl.log)"
done
DPA_FORCE_COMM=1 timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_rccl1.log 2>&1
echo "x3 rccl-1rank $(grep -o '"value": [0-9.]*' gpurun_out/bench_rccl1.log)"
timeout -k 10 200 python bench_resnet.py --batch 128 > gpurun_out/bench_resnet.log 2>&1
echo "resnet $(grep -o '"value": [0-9.]*' gpurun_out/bench_resnet.log)"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof.log 2>&1
echo prof-ok
