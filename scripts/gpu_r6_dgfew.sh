#!/bin/bash
# Round 6: data-gradient plans with fewer splits (the BN backward reduce then sums fewer slabs):
# layer 3 on one split, layer 5 on two; interleaved against the tuned table, parity on the winner set.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=distributed_pytorch_amd/tuning/ab
mkdir -p gpurun_out/dgfew
AB_ENVS="|DPA_TUNING_EXTRA=$T/ab_dg_l3.json|DPA_TUNING_EXTRA=$T/ab_dg_fewer.json" REPS=4 bash scripts/gpu_ab.sh 2>&1 | tee gpurun_out/dgfew_ab.log || exit 1
DPA_TUNING_EXTRA=$PWD/$T/ab_dg_fewer.json timeout -k 10 600 python -u -m pytest tests/test_parity256_gpu.py -q \
  --timeout 300 --timeout-method thread -k "fp32_grade or trained_state or loss_matches" > gpurun_out/dgfew_parity.log 2>&1
cp gpurun_out/parity256_errors.json gpurun_out/parity256_trained_errors.json gpurun_out/dgfew/
tail -1 gpurun_out/dgfew_parity.log
