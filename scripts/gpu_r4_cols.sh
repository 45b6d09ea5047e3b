# column-block forward BN: kernel tests, engine tests, VGG A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bn_gpu.py tests/test_ops_gpu.py tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_cols_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4_cols_tests.log; [ $rc -eq 0 ] || exit 1
REPS=3 AB_ENVS="DPA_BN_COLS=0 DPA_BN_COLS_BWD=0|DPA_BN_COLS=1 DPA_BN_COLS_BWD=0|DPA_BN_COLS=1 DPA_BN_COLS_BWD=1" bash scripts/gpu_ab.sh || exit 1
