set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
echo tests-ok
timeout -k 10 300 python tools/tune_convs.py --impls x3,bf16 > gpurun_out/tune.log 2>&1
cp distributed_pytorch_amd/tuning/mi355x.json gpurun_out/mi355x.json
echo tune-ok
timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/bench.log 2>&1
DPA_FORCE_COMM=1 timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_forcecomm.log 2>&1
tail -1 gpurun_out/bench.log gpurun_out/bench_forcecomm.log
