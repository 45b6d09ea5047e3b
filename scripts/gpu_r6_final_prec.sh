#!/bin/bash
# BN/ops tests, the parity suite, then the precision-gated in-step tuner (+ parity + A/B if it changes the table)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py tests/test_bn_wide_gpu.py tests/test_layer0_gpu.py tests/test_ops_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r6_bn_tests.log 2>&1; tail -3 gpurun_out/r6_bn_tests.log
timeout -k 10 400 python -u -m pytest tests/test_parity256_gpu.py -q --timeout 380 --timeout-method thread -k "fp32_grade or trained or loss" > gpurun_out/r6_parity.log 2>&1; grep -E "passed|failed|Error|assert" gpurun_out/r6_parity.log | tail -8
python - <<'PY'
import json
d = json.load(open("gpurun_out/parity256_trained_errors.json"))
for i in ("fp32", "x3", "h2"):
    t = d["torch_fp32"]["grads"]; f = d["fp32"]["grads"]
    r = sorted(e / max(t[n], 1e-12) for n, e in d[i]["grads"].items() if e is not None)
    r2 = sorted(e / max(f[n], 1e-12) for n, e in d[i]["grads"].items() if e is not None)
    print(i, "median vs torch32", round(r[len(r)//2], 3), "vs engine fp32", round(r2[len(r2)//2], 3))
PY
bash scripts/gpu_r6_tune.sh
