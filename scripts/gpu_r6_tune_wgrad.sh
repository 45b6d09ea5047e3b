#!/bin/bash
# Round 6: in-step re-tune of the weight-gradient plans (tools/tune_step.py, precision-gated) on the
# final forward / data-gradient plans; writes the candidate table to gpurun_out (not adopted here).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
cp distributed_pytorch_amd/tuning/mi355x.json gpurun_out/tuned_wgrad.json
timeout -k 10 720 python -u tools/tune_step.py --impl h2 --kinds wgrad --top 4 --reps 4 --gate-slack 0.5 \
  --out gpurun_out/tuned_wgrad.json > gpurun_out/tune_wgrad.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/tune_wgrad.log | grep -v "^  " | tail -15
exit $rc
