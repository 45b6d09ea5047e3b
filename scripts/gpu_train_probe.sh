#!/bin/bash
# Multi-rank training determinism probe (tests/ipc_train_worker.py): RUNS repetitions per mode.
set -o pipefail
mkdir -p gpurun_out/probe
k=0
for mode in ${MODES:-serial overlap}; do
  for rep in $(seq ${RUNS:-3}); do
    k=$((k+1))
    DPA_TRAIN_PROBE_MODE=$mode HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${W:-4} --master-addr 127.0.0.1 --master-port $((29600 + k)) tests/ipc_train_worker.py > gpurun_out/probe/${mode}_$rep.log 2>&1 || { tail -20 gpurun_out/probe/${mode}_$rep.log; exit 1; }
    echo "$mode $rep done"
  done
done
