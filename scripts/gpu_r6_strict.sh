#!/bin/bash
# Round-6: BN-tail A/B (fixed: no scratch), then the strict multi-rank oracle suite.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_bn_gpu.py -x -q --timeout 120 --timeout-method thread -k "backward" > gpurun_out/r6_bn_tests.log 2>&1 || { tail -40 gpurun_out/r6_bn_tests.log; exit 1; }
tail -1 gpurun_out/r6_bn_tests.log
AB_ENVS="DPA_BN_TAIL=0|DPA_BN_TAIL=1" REPS=3 STEPS=100 WARMUP=20 bash scripts/gpu_ab.sh || exit 1
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_multirank.log 2>&1 || { tail -60 gpurun_out/r6_multirank.log; exit 1; }
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r6_multirank.log | tail -40
