#!/bin/bash
# Round 6: the engine's fusion switches re-checked on the 64-chunk plans (interleaved, 100 steps).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
AB_ENVS="|DPA_FUSED_CONV0=0|DPA_BN_FUSED_MAX=4300000|DPA_FUSED_WGRAD0=0" REPS=3 bash scripts/gpu_ab.sh 2>&1 | tee gpurun_out/knobs_ab.log
