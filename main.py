"""Single-process VGG-11 / CIFAR-10 training (reference: main.py).

    python main.py [--synthetic] [--epochs 1] [--batch-size 256] [--device auto|cuda|cpu]
"""
from distributed_pytorch_amd.train import main_single

if __name__ == "__main__":
    main_single()
