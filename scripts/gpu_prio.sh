# wgrad-stream priority A/B (low vs normal), plus the single-rank sync tests and a trace of the winner.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 60 python -c "import torch; from distributed_pytorch_amd import _ext; print('prio range', _ext.require().stream_priority_range())"
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sync_modes or engine" > gpurun_out/prio_tests.log 2>&1 || { tail -30 gpurun_out/prio_tests.log; exit 1; }
tail -1 gpurun_out/prio_tests.log
for p in low normal low normal; do
  DPA_WGRAD_PRIO=$p timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_prio_$p.log 2>&1
  echo "x3 prio=$p $(grep -o '"value": [0-9.]*' gpurun_out/bench_prio_$p.log)"
done
for p in low normal; do
  DPA_WGRAD_PRIO=$p timeout -k 10 150 python bench.py --steps 50 --warmup 10 --impl bf16 > gpurun_out/bench_prio_bf16_$p.log 2>&1
  echo "bf16 prio=$p $(grep -o '"value": [0-9.]*' gpurun_out/bench_prio_bf16_$p.log)"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof.log 2>&1
echo prof-ok
