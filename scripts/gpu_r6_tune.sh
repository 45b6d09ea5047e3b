#!/bin/bash
# Round 6: in-step h2 plan tuning WITH the precision gate inside the tuner (tools/tune_step.py
# PrecisionGate), then the parity suite on the result and an interleaved A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tstep
timeout -k 10 900 python -u tools/tune_step.py --impl h2 --top ${TOP:-4} ${EXTRA:---per-split} --out gpurun_out/tstep/h2.json > gpurun_out/tstep/tune.log 2>&1 || { tail -20 gpurun_out/tstep/tune.log; exit 1; }
grep -E "precision|changed|start_step" gpurun_out/tstep/tune.log | cut -c1-400 | tail -30
[ -f gpurun_out/tstep/h2.json ] || { echo "no change"; exit 0; }
DPA_TUNING_EXTRA=gpurun_out/tstep/h2.json timeout -k 10 400 python -m pytest tests/test_parity256_gpu.py -q -x --timeout 380 \
  -k "h2" > gpurun_out/tstep/parity.log 2>&1 || { echo "parity suite failed:"; tail -8 gpurun_out/tstep/parity.log; exit 0; }
tail -1 gpurun_out/tstep/parity.log
REPS=${REPS:-4} STEPS=100 WARMUP=20 AB_ENVS="DPA_NO_TUNING=0|DPA_TUNING_EXTRA=gpurun_out/tstep/h2.json" bash scripts/gpu_ab.sh
