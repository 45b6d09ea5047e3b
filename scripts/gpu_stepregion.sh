# Fused SGD issued in the collective's comm region: sync-mode tests + 1-rank RCCL bench.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_layers_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sr_tests.log 2>&1 || { tail -30 gpurun_out/sr_tests.log; exit 1; }
tail -1 gpurun_out/sr_tests.log
for i in 1 2 3; do
  DPA_FORCE_COMM=1 timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/sr.log 2>&1
  echo "rccl1 $(grep -o '"value": [0-9.]*' gpurun_out/sr.log)"
done
timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/sr.log 2>&1
echo "null $(grep -o '"value": [0-9.]*' gpurun_out/sr.log)"
