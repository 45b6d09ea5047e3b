#!/bin/bash
# A/B: every kernel built without packed fp32 (variants/nopk/_C.so, DPA_NO_PACKED_FP32=1 build) vs the default build
set -o pipefail
AB_ENVS="DPA_STEP_HEALTH=1|DPA_EXT_SO=variants/nopk/_C.so" REPS=${REPS:-4} STEPS=100 WARMUP=20 bash scripts/gpu_ab.sh || exit 1
CFGS="nopk|DPA_EXT_SO=variants/nopk/_C.so" SECS=30 bash scripts/gpu_r6_replay.sh
