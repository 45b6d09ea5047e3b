#!/bin/bash
# W=4 (ranks sharing one GPU, peer-memory collectives): parameter checksums of the sync modes per
# conv implementation -- modes that reduce in rank order and scale in the update must agree bitwise.
set -o pipefail
mkdir -p gpurun_out/w4
for cfg in ${CFGS:-"allreduce:h2" "ddp:h2" "zero1:h2" "allreduce:x3" "ddp:x3"}; do
  m=${cfg%%:*}; i=${cfg##*:}
  timeout -k 10 200 python bench.py --gpus 4 --comm ipc --mode $m --steps 3 --warmup 2 --solo-steps 0 --diag-steps 1 --batch 64 --impl $i --launch-timeout 150 > gpurun_out/w4/${m}_$i.json 2>gpurun_out/w4/${m}_$i.err || exit 1
  echo "$cfg $(tail -1 gpurun_out/w4/${m}_$i.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["param_checksum"], d["replicas_identical"])')"
done
