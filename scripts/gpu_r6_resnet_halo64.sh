#!/bin/bash
# Round 6: ResNet-50 bf16 -- isolated A/B of the 64-channel-chunk halo tiles on the stride-1 3x3 convs,
# then an interleaved step A/B of the faster plans (DPA_GENERIC_TABLE = the table with them merged).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/resnet_halo64_ab.py > gpurun_out/resnet_halo64_ab.log 2>&1 || { tail -20 gpurun_out/resnet_halo64_ab.log; exit 1; }
cat gpurun_out/resnet_halo64_ab.log | grep -v amdgpu.ids
python - <<'PY'
import json
t = json.load(open("distributed_pytorch_amd/tuning/generic_mi355x.json"))
t.update(json.load(open("gpurun_out/resnet_halo64_cands.json")))
json.dump(t, open("gpurun_out/generic_new.json", "w"), indent=0, sort_keys=True)
PY
AB_ENVS="|DPA_GENERIC_TABLE=$PWD/gpurun_out/generic_new.json" BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=3 \
  bash scripts/gpu_ab.sh 2>&1 | tee gpurun_out/resnet_halo64_step_ab.log
