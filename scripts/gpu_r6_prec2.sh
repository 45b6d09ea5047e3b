#!/bin/bash
# fp64 BN statistics: BN / layer-0 / fused / eval tests, forward precision per layer, parity report,
# the parity suite, A/B vs the round-5 BN build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_bn_gpu.py tests/test_bn_wide_gpu.py tests/test_layer0_gpu.py tests/test_ops_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r6_bn_tests.log 2>&1 ; tail -3 gpurun_out/r6_bn_tests.log
timeout -k 10 200 python -u tools/step_check32.py > gpurun_out/step32.log 2>&1 || { tail -20 gpurun_out/step32.log; exit 1; }
cat gpurun_out/step32.log | grep -v amdgpu.ids
timeout -k 10 400 python -u tools/fwd_precision.py > gpurun_out/fwd_prec.log 2>&1 || { tail -20 gpurun_out/fwd_prec.log; exit 1; }
tail -11 gpurun_out/fwd_prec.log
timeout -k 10 400 python -u tools/parity_report.py > gpurun_out/r6_prec.log 2>&1 || { tail -20 gpurun_out/r6_prec.log; exit 1; }
grep -E "^(init|trained) " gpurun_out/r6_prec.log | cut -c1-600
bash scripts/gpu_r6_parity.sh || exit 1
AB_ENVS="DPA_STEP_HEALTH=1|DPA_EXT_SO=variants/f32bn/_C.so" REPS=${REPS:-3} STEPS=100 WARMUP=20 bash scripts/gpu_ab.sh
