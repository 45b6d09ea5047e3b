"""Data-parallel training, gradient sync mode B: per-tensor all-reduce then /W
(reference: main_all_reduce.py).

    python main_all_reduce.py --master-ip 127.0.0.1 --num-nodes 4 --rank $WORKER_RANK
"""
from distributed_pytorch_amd.train import main_cli

if __name__ == "__main__":
    main_cli("allreduce")
