# 64-column halo tiles (20/21): kernel tests, re-tune the layer-1 data gradient, bench x3/bf16.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "halo" > gpurun_out/halo64_tests.log 2>&1 || { tail -30 gpurun_out/halo64_tests.log; exit 1; }
tail -1 gpurun_out/halo64_tests.log
timeout -k 10 300 python tools/tune_convs.py --impls x3,bf16 --only "dgrad|256|16|64|128" > gpurun_out/tune64.log 2>&1
grep "dgrad\|sum_best" gpurun_out/tune64.log
cp distributed_pytorch_amd/tuning/mi355x.json gpurun_out/mi355x.json
for impl in x3 bf16; do
  timeout -k 10 150 python bench.py --steps 50 --warmup 10 --impl $impl > gpurun_out/bench64_$impl.log 2>&1
  echo "$impl $(grep -o '"value": [0-9.]*' gpurun_out/bench64_$impl.log)"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof.log 2>&1
echo prof-ok
