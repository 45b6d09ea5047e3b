"""Data-parallel training, gradient sync mode C: bucketed all-reduce overlapped with backward
(DistributedDataParallel semantics), launched by torchrun (reference: main_ddp.py, start_ddp.sh).

    torchrun --nproc_per_node=8 --nnodes=1 --master_addr=127.0.0.1 --master_port=6585 main_ddp.py
"""
from distributed_pytorch_amd.train import main_env

if __name__ == "__main__":
    main_env("ddp")
