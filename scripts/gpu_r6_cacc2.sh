#!/bin/bash
# Round 6 (per-chunk accumulation build): step A/B of the layer-3 one-split plan and the layer-3/4/5
# plans, and the parity suite on the latter.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=distributed_pytorch_amd/tuning/ab
mkdir -p gpurun_out/cacc_l345
AB_ENVS="|DPA_TUNING_EXTRA=$T/ab_l3_epi.json|DPA_TUNING_EXTRA=$T/ab_l345.json" REPS=4 bash scripts/gpu_ab.sh 2>&1 | tee gpurun_out/cacc_step_ab.log || exit 1
DPA_TUNING_EXTRA=$PWD/$T/ab_l345.json timeout -k 10 600 python -u -m pytest tests/test_parity256_gpu.py -q \
  --timeout 300 --timeout-method thread -k "fp32_grade or trained_state or loss_matches" > gpurun_out/cacc_l345_parity.log 2>&1
cp gpurun_out/parity256_errors.json gpurun_out/parity256_trained_errors.json gpurun_out/cacc_l345/
tail -1 gpurun_out/cacc_l345_parity.log
