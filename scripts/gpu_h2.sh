#!/bin/bash
# fp16-pair (h2) path: numerics tests, then an interleaved x3 / h2 bench A/B.
# STAGES: subset of "kern bn par bench" (default all)
set -o pipefail
mkdir -p gpurun_out/h2
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
ST=${STAGES:-"kern bn par bench"}
has() { [[ " $ST " == *" $1 "* ]]; }
if has kern; then timeout -k 10 600 $PT tests/test_kernels_gpu.py -k "fp16 or split or x3" > gpurun_out/h2/kern.log 2>&1 || exit 1; fi
if has bn; then timeout -k 10 300 $PT tests/test_bn_gpu.py > gpurun_out/h2/bn.log 2>&1 || exit 1; fi
if has par; then timeout -k 10 600 $PT tests/test_parity256_gpu.py tests/test_ops_gpu.py -k "h2 or parity" > gpurun_out/h2/par.log 2>&1 || exit 1; fi
if has bench; then
  for r in 1 2; do
    for impl in x3 h2; do
      timeout -k 10 240 python bench.py --steps 50 --warmup 10 --impl $impl > gpurun_out/h2/bench_${impl}_$r.json 2> gpurun_out/h2/bench_${impl}_$r.err || exit 1
    done
  done
fi
