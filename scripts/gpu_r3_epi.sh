# Conv-epilogue BN statistics: unit + ResNet tests, then a same-box ResNet-50 A/B.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_layers_gpu.py tests/test_parity256_gpu.py -k "epilogue or layers or resnet or parity" > gpurun_out/epi_tests.log 2>&1 || { tail -40 gpurun_out/epi_tests.log; exit 1; }
tail -3 gpurun_out/epi_tests.log
AB_ENVS="DPA_EPI_STATS=0|DPA_EPI_STATS=1" REPS=3 BENCH=bench_resnet.py STEPS=20 WARMUP=5 bash scripts/gpu_ab.sh
AB_ENVS="DPA_EPI_STATS=0|DPA_EPI_STATS=1" REPS=3 bash scripts/gpu_ab.sh
mv gpurun_out/rn_trace gpurun_out/rn_trace_prev 2>/dev/null || true
bash scripts/gpu_resnet_prof.sh
