#!/bin/bash
# Round 6: fewer split-K slabs for the small layers' convs (the one-launch BN sums fewer):
# layers 6/7 forward on 2 splits, layers 6/7 data gradient on 4, layer 4 data gradient on 2.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=distributed_pytorch_amd/tuning/ab
AB_ENVS="|DPA_TUNING_EXTRA=$T/ab_l67f.json|DPA_TUNING_EXTRA=$T/ab_l67d.json|DPA_TUNING_EXTRA=$T/ab_l4d.json" REPS=3 bash scripts/gpu_ab.sh 2>&1 | tee gpurun_out/small_ab.log
