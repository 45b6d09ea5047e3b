#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_health_gpu.py tests/test_signal_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6a_tests.log 2>&1 || { tail -40 gpurun_out/r6a_tests.log; exit 1; }
tail -2 gpurun_out/r6a_tests.log
bash scripts/gpu_replay.sh
