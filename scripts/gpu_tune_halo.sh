# New 4-wave 128x64 halo tiles: kernel tests, step-level retune of fprop/dgrad, bench.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "halo" -x -q --timeout 120 --timeout-method thread > gpurun_out/th_tests.log 2>&1 || { tail -40 gpurun_out/th_tests.log; exit 1; }
tail -1 gpurun_out/th_tests.log
timeout -k 10 150 python bench.py --steps 100 --warmup 20 > gpurun_out/th_bench0.log 2>&1 || { tail -20 gpurun_out/th_bench0.log; exit 1; }
tail -1 gpurun_out/th_bench0.log | cut -c1-200
timeout -k 10 700 python -u tools/tune_step.py --kinds fprop,dgrad --top 6 > gpurun_out/th_tune.log 2>&1 || { tail -30 gpurun_out/th_tune.log; exit 1; }
tail -2 gpurun_out/th_tune.log
cp distributed_pytorch_amd/tuning/mi355x.json gpurun_out/th_mi355x.json
timeout -k 10 150 python bench.py --steps 100 --warmup 20 > gpurun_out/th_bench1.log 2>&1 || { tail -20 gpurun_out/th_bench1.log; exit 1; }
tail -1 gpurun_out/th_bench1.log | cut -c1-200
