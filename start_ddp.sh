#!/usr/bin/env bash
# torchrun launcher for main_ddp.py (reference: start_ddp.sh).  One process per MI355X.
#   NNODES / NODE_RANK / MASTER_ADDR / MASTER_PORT / NPROC_PER_NODE may be overridden from the env
#   (the reference hard-codes --node_rank=0 and --nproc_per_node=1).
NPROC_PER_NODE=${NPROC_PER_NODE:-8}
NNODES=${NNODES:-1}
NODE_RANK=${NODE_RANK:-0}
MASTER_ADDR=${MASTER_ADDR:-127.0.0.1}
MASTER_PORT=${MASTER_PORT:-6585}
exec torchrun --nproc_per_node="$NPROC_PER_NODE" --nnodes="$NNODES" --node_rank="$NODE_RANK" \
  --master_addr="$MASTER_ADDR" --master_port="$MASTER_PORT" main_ddp.py "$@"
