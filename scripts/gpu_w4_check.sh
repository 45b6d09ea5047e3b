#!/bin/bash
# W ranks (default 4) sharing one GPU: parameter checksums of the sync modes, per conv implementation and
# environment.  CFGS: "mode:impl[:VAR=value,...]" items; COMM: ipc (default) | gloo | rccl.
set -o pipefail
mkdir -p gpurun_out/w4
n=0
for cfg in ${CFGS:-"allreduce:h2" "ddp:h2" "zero1:h2" "allreduce:x3" "ddp:x3"}; do
  IFS=: read -r m i e <<< "$cfg"; n=$((n+1))
  envs=$(echo "$e" | tr ',' ' ')
  env $envs timeout -k 10 200 python bench.py --gpus ${W:-4} --comm ${COMM:-ipc} --mode $m --steps ${STEPS:-3} --warmup 2 --solo-steps 0 --diag-steps 1 --batch 64 --impl $i ${XARGS:-} --launch-timeout 150 > gpurun_out/w4/run_$n.json 2>gpurun_out/w4/run_$n.err || exit 1
  echo "$cfg $(tail -1 gpurun_out/w4/run_$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["param_checksum"], d["replicas_identical"], d["final_loss"])')"
done
