#!/bin/bash
# Round 6: 64-channel-chunk halo tiles -- numerics (fp64) then the isolated A/B against the current plans.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "test_conv_halo or test_conv_epilogue_bn_stats" > gpurun_out/halo64_tests.log 2>&1 || { tail -30 gpurun_out/halo64_tests.log; exit 1; }
tail -3 gpurun_out/halo64_tests.log
timeout -k 10 300 python -u tools/halo64_ab.py --out gpurun_out/halo64_ab.json 2>&1 | tee gpurun_out/halo64_ab.log
