"""Measure the best (tile, split-K, position-major) for every conv call of the VGG training step
on this GPU and write distributed_pytorch_amd/tuning/mi355x.json (merged with existing entries).

    python tools/tune_convs.py [--impls fp32,x3,bf16] [--batch 256] [--only x3|dgrad|256|16|,...]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["DPA_NO_TUNING"] = "1"  # measure from scratch

from distributed_pytorch_amd.engine import VGGEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impls", default="fp32,x3,bf16")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--model", default="VGG11")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--only", default="", help="comma-separated conv_key substrings to re-tune (default: all)")
    ap.add_argument("--out", default=os.path.join(ROOT, "distributed_pytorch_amd", "tuning", "mi355x.json"))
    a = ap.parse_args()
    table = {}
    if os.path.exists(a.out):
        table = json.load(open(a.out))
    for impl in a.impls.split(","):
        e = VGGEngine(a.model, "cuda", max_batch=a.batch, impl=impl)
        x = torch.randn(a.batch, 32, 32, 4, device="cuda")
        x[..., 3] = 0
        e.x0.copy_(x)
        t = torch.randint(0, 10, (a.batch,), device="cuda")
        e.forward_backward(e.x0, t)
        torch.cuda.synchronize()
        res = e.autotune(a.batch, iters=a.iters, verbose=True, only=[o for o in a.only.split(",") if o] or None)
        table.update(res)
        tot = sum(v[3] for v in res.values())
        print(json.dumps({"impl": impl, "sum_best_conv_ms": round(tot, 4)}), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(table, f, indent=0, sort_keys=True)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
