set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python tools/diag_resnet_blocks.py > gpurun_out/diag_rn2.log 2>&1 || { tail -20 gpurun_out/diag_rn2.log; exit 1; }
cat gpurun_out/diag_rn2.log | tail -12
TESTS="tests/test_fused_gpu.py tests/test_parity256_gpu.py" bash scripts/gpu_iter.sh
