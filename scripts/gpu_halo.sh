# Halo kernels + wgrad stream: numerics, A/B bench, conv re-tune (x3, bf16), bench on the new table.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "halo" -x -q --timeout 120 --timeout-method thread > gpurun_out/halo_tests.log 2>&1 || { tail -40 gpurun_out/halo_tests.log; exit 1; }
tail -1 gpurun_out/halo_tests.log
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "wgrad_stream or engine_step or sync_modes" -x -q --timeout 120 --timeout-method thread > gpurun_out/ops_tests.log 2>&1 || { tail -40 gpurun_out/ops_tests.log; exit 1; }
tail -1 gpurun_out/ops_tests.log
for ws in 0 1; do
  DPA_WGRAD_STREAM=$ws timeout -k 10 120 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_ws$ws.log 2>&1
  echo "ws=$ws $(grep -o '"value": [0-9.]*' gpurun_out/bench_ws$ws.log)"
done
if [ "${TUNE:-1}" = 1 ]; then
  timeout -k 10 600 python -u tools/tune_convs.py --impls x3,bf16 > gpurun_out/tune.log 2>&1
  cp distributed_pytorch_amd/tuning/mi355x.json gpurun_out/mi355x.json
  grep sum_best gpurun_out/tune.log
  timeout -k 10 120 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_tuned.log 2>&1
  echo "tuned x3 $(grep -o '"value": [0-9.]*' gpurun_out/bench_tuned.log)"
  timeout -k 10 120 python bench.py --steps 30 --warmup 10 --impl bf16 > gpurun_out/bench_tuned_bf16.log 2>&1
  echo "tuned bf16 $(grep -o '"value": [0-9.]*' gpurun_out/bench_tuned_bf16.log)"
fi
