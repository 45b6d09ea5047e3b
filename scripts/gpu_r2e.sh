set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 120 python tools/micro_bn_small.py > gpurun_out/micro_bn_small.log 2>&1 || { tail -20 gpurun_out/micro_bn_small.log; exit 1; }
cat gpurun_out/micro_bn_small.log
TESTS="tests/test_fused_gpu.py" bash scripts/gpu_iter.sh
