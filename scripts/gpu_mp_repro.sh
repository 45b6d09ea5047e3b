#!/bin/bash
# Multi-process reproducibility probe (tools/mp_repro.py) then W-rank training checksums.
set -o pipefail
mkdir -p gpurun_out/mp
timeout -k 10 400 python -u tools/mp_repro.py --procs ${P:-4} --seconds ${SECS:-12} --mode ${MODES:-fill,conv0,conv0alt,signal} > gpurun_out/mp/probe.jsonl 2> gpurun_out/mp/probe.err || { tail -20 gpurun_out/mp/probe.err; exit 1; }
cat gpurun_out/mp/probe.jsonl | python -c 'import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d["mode"], "bad_total", d["bad_total"], [ (r["iters"], r["bad"]) for r in d["rows"]])'
for k in $(seq 1 ${RUNS:-0}); do
  timeout -k 10 200 python bench.py --gpus 4 --comm gloo --mode ddp --steps 3 --warmup 2 --solo-steps 0 --diag-steps 0 --batch 64 --comm-tune off --launch-timeout 150 > gpurun_out/mp/w4_$k.json 2>gpurun_out/mp/w4_$k.err || exit 1
  tail -1 gpurun_out/mp/w4_$k.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("w4", d["param_checksum"], d["replicas_identical"])'
done
