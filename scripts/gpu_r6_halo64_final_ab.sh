#!/bin/bash
# Round 6: interleaved step A/B of the adopted 64-chunk plans against the previous ones.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
AB_ENVS="DPA_TUNING_EXTRA=distributed_pytorch_amd/tuning/ab/ab_old_r6.json|DPA_AB_NEW=1" REPS=4 bash scripts/gpu_ab.sh 2>&1 | tee gpurun_out/halo64_final_ab.log
