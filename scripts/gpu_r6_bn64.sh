#!/bin/bash
# BN backward precision: fp64 sums + centred dz coefficients.  BN / layer-0 / ops kernel tests, the
# parity suite (random init + trained state), A/B vs the round-5 BN build (variants/f32bn)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_bn_gpu.py tests/test_bn_wide_gpu.py tests/test_layer0_gpu.py tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_bn_tests.log 2>&1 || { tail -30 gpurun_out/r6_bn_tests.log; exit 1; }
tail -1 gpurun_out/r6_bn_tests.log
bash scripts/gpu_r6_parity.sh || exit 1
AB_ENVS="DPA_STEP_HEALTH=1|DPA_EXT_SO=variants/f32bn/_C.so" REPS=${REPS:-3} STEPS=100 WARMUP=20 bash scripts/gpu_ab.sh
