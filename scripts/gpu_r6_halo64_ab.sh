#!/bin/bash
# Round 6: step A/B of the 64-channel-chunk halo plans (tuning/ab/halo64_all.json) and the parity
# suite with them installed.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
X=distributed_pytorch_amd/tuning/ab/halo64_all.json
AB_ENVS="|DPA_TUNING_EXTRA=$X" REPS=4 bash scripts/gpu_ab.sh 2>&1 | tee gpurun_out/halo64_step_ab.log || exit 1
DPA_TUNING_EXTRA=$PWD/$X timeout -k 10 600 python -u -m pytest tests/test_parity256_gpu.py -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/halo64_parity.log 2>&1; rc=$?
tail -15 gpurun_out/halo64_parity.log
exit $rc
