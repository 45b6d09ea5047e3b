# HIP-graph step: parity test, host enqueue tool, interleaved bench A/B (eager vs graph).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "graphed" > gpurun_out/graph_tests.log 2>&1 || { tail -40 gpurun_out/graph_tests.log; exit 1; }
tail -1 gpurun_out/graph_tests.log
timeout -k 10 120 python tools/host_overhead.py --graph > gpurun_out/host_graph.log 2>&1; tail -1 gpurun_out/host_graph.log
timeout -k 10 120 python tools/host_overhead.py > gpurun_out/host_eager.log 2>&1; tail -1 gpurun_out/host_eager.log
for i in 1 2; do
  for gmode in off on; do
    timeout -k 10 150 python bench.py --steps 50 --warmup 10 --graph $gmode > gpurun_out/bench_graph_$gmode.log 2>&1
    echo "x3 graph=$gmode $(grep -o '"value": [0-9.]*' gpurun_out/bench_graph_$gmode.log)"
  done
done
for gmode in off on; do
  timeout -k 10 150 python bench.py --steps 50 --warmup 10 --graph $gmode --impl bf16 > gpurun_out/bench_graph_bf16_$gmode.log 2>&1
  echo "bf16 graph=$gmode $(grep -o '"value": [0-9.]*' gpurun_out/bench_graph_bf16_$gmode.log)"
done
