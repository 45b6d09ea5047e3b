#!/bin/bash
# Peer-memory all-reduce stress (tests/ipc_stress_worker.py) at W ranks on one GPU.
set -o pipefail
mkdir -p gpurun_out/stress
for W in ${WORLDS:-4 8}; do
  HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port $((29500 + W)) tests/ipc_stress_worker.py > gpurun_out/stress/w$W.log 2>&1
  echo "W=$W rc=$?"; grep '^{' gpurun_out/stress/w$W.log
done
