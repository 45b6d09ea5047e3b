"""Data-parallel training, DDP semantics, launched with the mode-A/B CLI (reference: main_part3.py).

    python main_part3.py --master-ip 127.0.0.1 --num-nodes 4 --rank $WORKER_RANK
"""
from distributed_pytorch_amd.train import main_cli

if __name__ == "__main__":
    main_cli("ddp")
