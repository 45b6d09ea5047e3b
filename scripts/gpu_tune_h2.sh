#!/bin/bash
# Measure the fp16-pair (h2) conv plans, merge them into the tuning table, bench h2 on them.
set -o pipefail
mkdir -p gpurun_out/tune
timeout -k 10 900 python -u tools/tune_convs.py --impls h2 --out gpurun_out/tune/h2.json > gpurun_out/tune/tune.log 2>&1 &&
python - <<'PY' &&
import json
p = "distributed_pytorch_amd/tuning/mi355x.json"
t = json.load(open(p)); t.update(json.load(open("gpurun_out/tune/h2.json")))
json.dump(t, open(p, "w"), indent=0, sort_keys=True)
PY
for r in 1 2; do
  timeout -k 10 240 python bench.py --steps 50 --warmup 10 --impl h2 > gpurun_out/tune/bench_h2_$r.json 2> gpurun_out/tune/bench_h2_$r.err || exit 1
done
