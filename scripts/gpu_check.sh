# GPU validation pass: kernel/ops tests, conv re-tune, bench, kernel profile.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
if [ "${TUNE:-1}" = 1 ]; then
  timeout -k 10 400 python tools/tune_convs.py --impls x3,bf16 > gpurun_out/tune.log 2>&1
  cp distributed_pytorch_amd/tuning/mi355x.json gpurun_out/mi355x.json
  grep sum_best gpurun_out/tune.log
fi
timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/bench.log 2>&1
grep metric gpurun_out/bench.log | cut -c 1-260
timeout -k 10 200 python bench.py --steps 30 --warmup 10 --impl bf16 > gpurun_out/bench_bf16.log 2>&1
grep metric gpurun_out/bench_bf16.log | cut -c 1-260
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof.log 2>&1
echo prof-ok
