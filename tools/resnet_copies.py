"""Where the ResNet-50 step's device copies come from: one eager training step of bench_resnet's
model under torch.profiler, aten::copy_ / clone / contiguous grouped by the innermost call site in
this package (file:line), with counts and device time.

    python tools/resnet_copies.py [--batch 128]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_amd.models.resnet import resnet50  # noqa: E402
from distributed_pytorch_amd.parallel.ddp import DistributedDataParallel, FlatSGD  # noqa: E402
from distributed_pytorch_amd.parallel.launch import init_env  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    ctx = init_env(comm="rccl")
    dev = ctx.device
    torch.manual_seed(1)
    model = resnet50(1000, "bf16").to(dev)
    ddp = DistributedDataParallel(model, ctx.comm, bucket_mb=25.0)
    opt = FlatSGD(ddp, lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(a.batch, 224, 224, 3, device=dev)
    t = torch.randint(0, 1000, (a.batch,), device=dev)
    one = torch.ones((), device=dev)

    def step():
        opt.zero_grad()
        loss = ddp(x, t)
        loss.backward(one)
        opt.step(ddp.finish())

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    allr = prof.key_averages()
    print(f"{len(allr)} distinct ops; most frequent:", flush=True)
    for r in sorted(allr, key=lambda r: -r.count)[:25]:
        print(f"{r.count:5d}  {r.key[:90]}")
    rows = [r for r in prof.key_averages(group_by_stack_n=6)
            if any(w in r.key.lower() for w in ("copy", "memcpy", "clone", "contiguous", "fill", "zero_"))]
    for r in sorted(rows, key=lambda r: -r.count)[:40]:
        dev_us = getattr(r, "device_time_total", 0.0) or getattr(r, "cuda_time_total", 0.0)
        stack = [f for f in (r.stack or []) if "site-packages" not in f and "dist-packages" not in f]
        print(f"{r.count:5d} {dev_us:9.1f} us  {r.key[:50]}")
        for f in stack[:4]:
            print(f"          {f}")

if __name__ == "__main__":
    main()
