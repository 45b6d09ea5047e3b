#!/bin/bash
# Round 6: per-chunk accumulation in the fp16-pair 64-channel halo tiles -- fp64 tests, parity suite on
# the tuned table and with the layer-3 one-split plan, isolated timing.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/cacc gpurun_out/cacc_l3
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "test_conv_halo or test_conv_epilogue_bn_stats" > gpurun_out/cacc_tests.log 2>&1 || { tail -30 gpurun_out/cacc_tests.log; exit 1; }
tail -1 gpurun_out/cacc_tests.log
timeout -k 10 600 python -u -m pytest tests/test_parity256_gpu.py -q --timeout 300 --timeout-method thread \
  -k "fp32_grade or trained_state or loss_matches" > gpurun_out/cacc_parity.log 2>&1
cp gpurun_out/parity256_errors.json gpurun_out/parity256_trained_errors.json gpurun_out/cacc/
tail -1 gpurun_out/cacc_parity.log
DPA_TUNING_EXTRA=$PWD/distributed_pytorch_amd/tuning/ab/ab_l3_epi.json timeout -k 10 600 python -u -m pytest tests/test_parity256_gpu.py -q \
  --timeout 300 --timeout-method thread -k "fp32_grade or trained_state or loss_matches" > gpurun_out/cacc_l3_parity.log 2>&1
cp gpurun_out/parity256_errors.json gpurun_out/parity256_trained_errors.json gpurun_out/cacc_l3/
tail -1 gpurun_out/cacc_l3_parity.log
timeout -k 10 300 python -u tools/halo64_ab.py --rounds 3 --out gpurun_out/cacc_ab.json 2>&1 | grep -v amdgpu.ids | tee gpurun_out/cacc_ab.log
