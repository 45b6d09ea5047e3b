"""ATen-level breakdown of the ResNet-50 generic-path training step (torch.profiler): which
torch ops (copies, adds, pooling...) run around the native kernels, how often and for how long.

    python tools/resnet_ops.py [--batch 128] [--steps 3]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_amd.models.resnet import resnet50  # noqa: E402
from distributed_pytorch_amd.parallel.ddp import DistributedDataParallel, FlatSGD  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    ddp = DistributedDataParallel(resnet50(1000, "bf16").to(dev))
    opt = FlatSGD(ddp, lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(a.batch, 224, 224, 3, device=dev)
    t = torch.randint(0, 1000, (a.batch,), device=dev)

    def step():
        opt.zero_grad()
        F.cross_entropy(ddp(x), t).backward()
        opt.step(ddp.finish())

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts) as prof:
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_device_time_total", row_limit=40, max_name_column_width=60))


if __name__ == "__main__":
    main()
