#!/bin/bash
# In-step conv plan tuning for h2 (tools/tune_step.py), then the precision gate (the parity suite's
# fp32-grade gradient check on the candidate entries) and an interleaved A/B of the result.
#   EXTRA=--per-split bash scripts/gpu_tune_step_h2.sh
set -o pipefail
mkdir -p gpurun_out/tstep
timeout -k 10 700 python -u tools/tune_step.py --impl h2 --top ${TOP:-4} ${EXTRA:-} --out gpurun_out/tstep/h2.json > gpurun_out/tstep/tune.log 2>&1 || { tail -20 gpurun_out/tstep/tune.log; exit 1; }
tail -2 gpurun_out/tstep/tune.log
[ -f gpurun_out/tstep/h2.json ] || { echo "no change"; exit 0; }
DPA_TUNING_EXTRA=gpurun_out/tstep/h2.json timeout -k 10 300 python -m pytest tests/test_parity256_gpu.py -q -x --timeout 280 \
  -k "fp32_grade and h2" > gpurun_out/tstep/parity.log 2>&1 || { echo "candidate rejected on precision:"; tail -5 gpurun_out/tstep/parity.log; exit 0; }
echo "precision gate passed"
REPS=${REPS:-4} STEPS=100 WARMUP=20 AB_ENVS="DPA_NO_TUNING=0|DPA_TUNING_EXTRA=gpurun_out/tstep/h2.json" bash scripts/gpu_ab.sh
