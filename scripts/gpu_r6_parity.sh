#!/bin/bash
# the parity suite (random init and trained state) on the current tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_parity256_gpu.py -v --timeout 450 --timeout-method thread -k "fp32_grade or trained or loss" > gpurun_out/r6_parity.log 2>&1; rc=$?
grep -E "PASS|FAIL|assert|passed|failed" gpurun_out/r6_parity.log | cut -c1-300 | tail -30
python - <<'PY'
import json
for f in ("gpurun_out/parity256_errors.json", "gpurun_out/parity256_trained_errors.json"):
    try:
        d = json.load(open(f))
    except Exception as e:
        print(f, e); continue
    tref = d["torch_fp32"]["grads"]
    for impl in ("fp32", "x3", "h2"):
        if impl not in d: continue
        r = sorted(e / max(tref[n], 1e-12) for n, e in d[impl]["grads"].items() if e is not None)
        print(f, impl, "median ratio", round(r[len(r)//2], 3), "max", round(r[-1], 2))
PY
[ $rc -le 1 ] || exit $rc  # (a failing test is a result; a timeout or crash ends the call)
