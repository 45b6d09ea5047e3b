#!/bin/bash
# Round 6: interleaved step A/B: current table | gate-passing data-gradient plans | all 64-chunk plans.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=distributed_pytorch_amd/tuning/ab
AB_ENVS="|DPA_TUNING_EXTRA=$T/halo64_dgrad.json|DPA_TUNING_EXTRA=$T/halo64_all.json" REPS=4 bash scripts/gpu_ab.sh 2>&1 | tee gpurun_out/halo64_step_ab2.log
