"""Stock PyTorch-ROCm eager baseline for the reference workload on one MI355X.

The reference's own training step (main.py:31-37: zero_grad, forward, CE, backward,
SGD(0.1, 0.9, 1e-4)) on model.VGG11 — re-created here with stock torch.nn modules (MIOpen convs,
no custom kernels) — timed at batch 256.  This is the bar SURVEY §6 says the framework must beat.

    python tools/torch_baseline.py --steps 30 --warmup 10
    python tools/torch_baseline.py --model resnet50 --batch 128 --modes bf16_cl   # stress config
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn as nn

CFG = [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"]


def vgg11():
    layers, c = [], 3
    for v in CFG:
        if v == "M":
            layers.append(nn.MaxPool2d(2, 2))
        else:
            layers += [nn.Conv2d(c, v, 3, 1, 1, bias=True), nn.BatchNorm2d(v), nn.ReLU(inplace=True)]
            c = v

    class V(nn.Module):
        def __init__(self):
            super().__init__()
            self.layers = nn.Sequential(*layers)
            self.fc1 = nn.Linear(512, 10)

        def forward(self, x):
            y = self.layers(x)
            return self.fc1(y.view(y.size(0), -1))

    return V()


def run(mode, steps, warmup, batch, model="vgg11"):
    torch.manual_seed(1)
    if model == "resnet50":
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from distributed_pytorch_amd.models.resnet import ResNetRef

        m = ResNetRef([3, 4, 6, 3], 1000).cuda()
        x = torch.randn(batch, 3, 224, 224, device="cuda")
        t = torch.randint(0, 1000, (batch,), device="cuda")
    else:
        m = vgg11().cuda()
        x = torch.randn(batch, 3, 32, 32, device="cuda")
        t = torch.randint(0, 10, (batch,), device="cuda")
    if mode in ("channels_last", "bf16_cl"):
        m = m.to(memory_format=torch.channels_last)
        x = x.to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    crit = nn.CrossEntropyLoss()

    def step():
        opt.zero_grad()
        if mode in ("bf16", "bf16_cl"):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = m(x)
                loss = crit(out.float(), t)
        else:
            out = m(x)
            loss = crit(out, t)
        loss.backward()
        opt.step()
        return loss

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return {"model": model, "mode": mode, "batch": batch, "ms_per_step": dt * 1e3, "img_per_s": batch / dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--modes", default="fp32,channels_last,bf16")
    ap.add_argument("--model", default="vgg11", choices=["vgg11", "resnet50"])
    a = ap.parse_args()
    for mode in a.modes.split(","):
        print(json.dumps(run(mode, a.steps, a.warmup, a.batch, a.model)), flush=True)


if __name__ == "__main__":
    main()
