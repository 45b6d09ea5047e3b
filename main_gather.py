"""Data-parallel training, gradient sync mode A: gather to rank 0 → mean → broadcast
(reference: main_gather.py).

    python main_gather.py --master-ip 127.0.0.1 --num-nodes 4 --rank $WORKER_RANK
"""
from distributed_pytorch_amd.train import main_cli

if __name__ == "__main__":
    main_cli("gather")
