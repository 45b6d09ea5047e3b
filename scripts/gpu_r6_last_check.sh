#!/bin/bash
# Round 6: last check of the committed tree's in-tree build: smoke, kernel/engine subset, driver-style bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/last
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/last/smoke.log 2>&1 || { tail -20 gpurun_out/last/smoke.log; exit 1; }
tail -1 gpurun_out/last/smoke.log
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_layer0_gpu.py tests/test_parity256_gpu.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/last/tests.log 2>&1 || { tail -20 gpurun_out/last/tests.log; exit 1; }
tail -1 gpurun_out/last/tests.log
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > gpurun_out/last/bench.json 2> gpurun_out/last/bench.err || { tail -20 gpurun_out/last/bench.err; exit 1; }
tail -1 gpurun_out/last/bench.json | cut -c1-220
