# Post-forward BN-buffer broadcast: sync-mode tests through 1-rank RCCL, interleaved A/B.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sync_modes or graphed" > gpurun_out/bb_tests.log 2>&1 || { tail -30 gpurun_out/bb_tests.log; exit 1; }
tail -1 gpurun_out/bb_tests.log
for i in 1 2; do
  for v in post pre; do
    DPA_BUF_BCAST=$v DPA_FORCE_COMM=1 timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/bb.log 2>&1
    echo "rccl1 bufbcast=$v $(grep -o '"value": [0-9.]*' gpurun_out/bb.log)"
  done
done
timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/bb.log 2>&1
echo "null $(grep -o '"value": [0-9.]*' gpurun_out/bb.log)"
