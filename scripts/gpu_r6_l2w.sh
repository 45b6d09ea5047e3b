#!/bin/bash
# Round 6: the in-step tuner's layer-2 weight-gradient plan (tile 4, 32 splits) against the table's.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
AB_ENVS="|DPA_TUNING_EXTRA=distributed_pytorch_amd/tuning/ab/ab_l2w.json" REPS=4 bash scripts/gpu_ab.sh 2>&1 | tee gpurun_out/l2w_ab.log
