"""Training-trajectory check: the engine's conv arithmetics against stock PyTorch fp32 over many steps.

The same VGG-11 (seed-1 init, models/vgg.py), the same augmented batches (DeviceLoader, same seeds)
and SGD(lr, 0.9, 1e-4) are trained once per engine implementation (h2 / x3 / fp32 MFMA) and once
with stock torch eager fp32 (MIOpen convs, torch.optim.SGD, TF32 off).  Prints one JSON line: the
loss every ``--every`` steps of each run and, at the end, each engine run's per-tensor relative
L2 distance of the parameters from the torch run (max and median over the 58 state_dict tensors).
An fp32-grade implementation lands as close to the torch run as the exact-fp32 engine does (the
residual is summation order, amplified by training); a lower-precision one drifts further.

    python tools/train_curve.py [--steps 300] [--every 10] [--impls h2,x3,fp32] [--batch 256] [--lr 0.1]
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_pytorch_amd.data import DeviceLoader, ShardSampler, synthetic_cifar  # noqa: E402
from distributed_pytorch_amd.engine import VGGEngine  # noqa: E402
from distributed_pytorch_amd.models.vgg import VGG  # noqa: E402


def batches(ds, batch, dev):
    ld = DeviceLoader(ds, batch, dev, sampler=ShardSampler(len(ds), 1, 0, shuffle=True, seed=0), train=True,
                      seed=7919, drop_last=True)
    ep = 0
    while True:
        ld.set_epoch(ep)
        for x, t in ld:
            yield x, t
        ep += 1


def run_engine(impl, ds, a, dev):
    e = VGGEngine("VGG11", dev, max_batch=a.batch, impl=impl, lr=a.lr)
    e.init_parameters(seed=1)
    it = batches(ds, a.batch, dev)
    losses = []
    for s in range(a.steps):
        x, t = next(it)
        e.forward_backward(x, t)
        e.sgd_step()
        e.finish_step()
        if s % a.every == 0 or s == a.steps - 1:
            losses.append(round(float(e.loss.item()), 6))
    e.check_signals()
    return losses, {k: v.detach().float().cpu() for k, v in e.state_dict().items()}


def run_torch(ds, a, dev):
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.manual_seed(1)
    m = VGG("VGG11", 10).to(dev)
    opt = torch.optim.SGD(m.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4)
    it = batches(ds, a.batch, dev)
    losses = []
    for s in range(a.steps):
        x, t = next(it)
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(m(x[..., :3].permute(0, 3, 1, 2).contiguous()), t)
        loss.backward()
        opt.step()
        if s % a.every == 0 or s == a.steps - 1:
            losses.append(round(float(loss.item()), 6))
    return losses, {k: v.detach().float().cpu() for k, v in m.state_dict().items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--every", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--impls", default="h2,x3,fp32")
    ap.add_argument("--lr", type=float, default=0.1)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ds = synthetic_cifar(50000, 0)
    ref_loss, ref_sd = run_torch(ds, a, dev)
    out = {"steps": a.steps, "every": a.every, "batch": a.batch, "lr": a.lr, "torch_fp32_loss": ref_loss, "runs": {}}
    for impl in a.impls.split(","):
        losses, sd = run_engine(impl, ds, a, dev)
        rel = []
        for k, v in ref_sd.items():
            if not v.is_floating_point() or k not in sd:
                continue
            w = sd[k].reshape(v.shape) if sd[k].numel() == v.numel() else None
            if w is None:
                continue
            rel.append(float((w - v).norm() / max(float(v.norm()), 1e-30)))
        out["runs"][impl] = {"loss": losses, "param_rel_l2_max": max(rel), "param_rel_l2_median": statistics.median(rel),
                             "tensors": len(rel)}
        print(json.dumps({"impl": impl, "final_loss": losses[-1], "torch_final_loss": ref_loss[-1],
                          "param_rel_l2_max": max(rel)}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
