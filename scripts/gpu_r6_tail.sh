#!/bin/bash
# Round-6: BN tests (tail finalize), replay (default), then interleaved A/B of DPA_BN_TAIL.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "bn or conv0 or first" > gpurun_out/r6_bn_tests.log 2>&1 || { tail -40 gpurun_out/r6_bn_tests.log; exit 1; }
tail -1 gpurun_out/r6_bn_tests.log
CFGS="${RCFGS:-default|}" SECS=40 bash scripts/gpu_r6_replay.sh || exit 1
AB_ENVS="DPA_BN_TAIL=0|DPA_BN_TAIL=1" REPS=${REPS:-3} STEPS=100 WARMUP=20 bash scripts/gpu_ab.sh || exit 1
