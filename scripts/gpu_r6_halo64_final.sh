#!/bin/bash
# Round 6: the adopted 64-chunk plans -- interleaved step A/B against the previous plans
# (tuning/ab/ab_old_r6.json), then the parity suite and the fused/layer tests on the new table.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
AB_ENVS="DPA_TUNING_EXTRA=distributed_pytorch_amd/tuning/ab/ab_old_r6.json|DPA_AB_NEW=1" REPS=4 bash scripts/gpu_ab.sh 2>&1 | tee gpurun_out/halo64_final_ab.log || exit 1
timeout -k 10 600 python -u -m pytest tests/test_parity256_gpu.py tests/test_engine_cpu.py -x -q --timeout 300 \
  --timeout-method thread -m gpu > gpurun_out/halo64_final_parity.log 2>&1; rc=$?
tail -3 gpurun_out/halo64_final_parity.log
exit $rc
