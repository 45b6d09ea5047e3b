#!/bin/bash
# conv0 two-channel variant: layer-0 tests both ways, the fused-kernel tests, A/B, replay under load
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="tests/test_layer0_gpu.py tests/test_fused_gpu.py tests/test_ops_gpu.py"
timeout -k 10 300 python -u -m pytest $T -q --timeout 200 --timeout-method thread > gpurun_out/c0_tests_a.log 2>&1; tail -2 gpurun_out/c0_tests_a.log
DPA_CONV0_CH2=1 timeout -k 10 300 python -u -m pytest $T -q --timeout 200 --timeout-method thread > gpurun_out/c0_tests_b.log 2>&1; tail -2 gpurun_out/c0_tests_b.log
AB_ENVS="DPA_CONV0_CH2=0|DPA_CONV0_CH2=1" REPS=4 STEPS=100 WARMUP=20 bash scripts/gpu_ab.sh || exit 1
CFGS="ch2|DPA_CONV0_CH2=1" SECS=30 bash scripts/gpu_r6_replay.sh
