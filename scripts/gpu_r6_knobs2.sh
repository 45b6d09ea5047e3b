#!/bin/bash
# Round 6: one-launch BN knobs on the final plans (row blocks per slice; forward size threshold).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
AB_ENVS="|DPA_BN_FUSED_RMAX=32|DPA_BN_FUSED_RMAX=128|DPA_BN_FUSED_MAX=600000" REPS=3 bash scripts/gpu_ab.sh 2>&1 | tee gpurun_out/knobs2_ab.log
