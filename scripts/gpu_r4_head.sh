# ResNet head backward prep: 16 rows' loads in flight; tests + trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_layers_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4head_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4head_tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/gpu_r4_rnprof.sh || exit 1
