#!/bin/bash
# IPC live-agreement and forced-disagreement tests, then the null-comm / 1-rank RCCL traces.
set -o pipefail
mkdir -p gpurun_out/ipc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multirank_gpu.py -k "live_agreement or forced_disagreement" > gpurun_out/ipc/checks.log 2>&1 || exit 1
if [ "${TRACES:-1}" = 1 ]; then
  TAG=r5null bash scripts/gpu_profile.sh && DPA_FORCE_COMM=1 TAG=r5rccl bash scripts/gpu_profile.sh
fi
