#!/bin/bash
# In-step conv plan tuning for h2 (tools/tune_step.py), then an interleaved A/B of the result.
set -o pipefail
mkdir -p gpurun_out/tstep
timeout -k 10 700 python -u tools/tune_step.py --impl h2 --top ${TOP:-4} ${EXTRA:-} --out gpurun_out/tstep/h2.json > gpurun_out/tstep/tune.log 2>&1 || { tail -20 gpurun_out/tstep/tune.log; exit 1; }
tail -2 gpurun_out/tstep/tune.log
[ -f gpurun_out/tstep/h2.json ] || { echo "no change"; exit 0; }
REPS=3 STEPS=50 WARMUP=10 AB_ENVS="DPA_NO_TUNING=0|DPA_TUNING_EXTRA=gpurun_out/tstep/h2.json" bash scripts/gpu_ab.sh
