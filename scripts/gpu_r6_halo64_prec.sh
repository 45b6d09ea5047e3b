#!/bin/bash
# Round 6: parity-suite errors with the current table (baseline) for comparison with the
# 64-channel-chunk halo plans (gpu_r6_halo64_ab.sh ran the suite with them).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/base
timeout -k 10 600 python -u -m pytest tests/test_parity256_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "test_all_gradients_fp32_grade or test_parity_at_trained_state" > gpurun_out/base/parity.log 2>&1; rc=$?
cp gpurun_out/parity256_errors.json gpurun_out/parity256_trained_errors.json gpurun_out/base/ 2>/dev/null
tail -3 gpurun_out/base/parity.log
exit $rc
