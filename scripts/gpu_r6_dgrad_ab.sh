#!/bin/bash
# Round 6: which 64-chunk data-gradient plans pay in the step: all new | old dgrad plans | old but layer 1.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=distributed_pytorch_amd/tuning/ab
AB_ENVS="|DPA_TUNING_EXTRA=$T/ab_olddgrad_r6.json|DPA_TUNING_EXTRA=$T/ab_olddgrad_but_l1_r6.json" REPS=4 bash scripts/gpu_ab.sh 2>&1 | tee gpurun_out/dgrad_ab.log
