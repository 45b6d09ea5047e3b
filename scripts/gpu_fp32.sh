set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python tools/tune_convs.py --impls fp32 > gpurun_out/tune_fp32.log 2>&1
cp distributed_pytorch_amd/tuning/mi355x.json gpurun_out/mi355x.json
grep sum_best gpurun_out/tune_fp32.log
timeout -k 10 200 python bench.py --steps 30 --warmup 10 --impl fp32 | cut -c 1-200
