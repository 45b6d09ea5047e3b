#!/bin/bash
# Round 6: 64-channel-chunk halo tiles -- fp64 kernel tests, then the gated adoption of the plans
# (tools/adopt_plans.py), then the isolated A/B over every eligible call (tools/halo64_ab.py --all).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "test_conv_halo or test_conv_epilogue_bn_stats" > gpurun_out/halo64_tests.log 2>&1 || { tail -30 gpurun_out/halo64_tests.log; exit 1; }
tail -1 gpurun_out/halo64_tests.log
timeout -k 10 900 python -u tools/adopt_plans.py --cands distributed_pytorch_amd/tuning/candidates_r6_halo64.json --impl h2 \
  --write --out gpurun_out/adopted_plans.json --log gpurun_out/adopt_plans.json > gpurun_out/adopt_plans.log 2>&1 || { tail -20 gpurun_out/adopt_plans.log; exit 1; }
tail -2 gpurun_out/adopt_plans.log
timeout -k 10 300 python -u tools/halo64_ab.py --all --only "|4|256|512,|2|512|512,|4|512|512" --out gpurun_out/halo64_ab_all.json > gpurun_out/halo64_ab_all.log 2>&1
tail -8 gpurun_out/halo64_ab_all.log
