"""Per-shape conv timing for the ResNet-50 training step (batch 128, 224x224, bf16): this
framework's kernels (generic autograd path, tuned table) vs stock torch (MIOpen, channels_last)
vs a plain hipBLASLt GEMM (torch.matmul) for the 1x1 convs.  Times are fprop + dgrad + wgrad,
multiplied by how often the shape occurs in the network.

    python tools/resnet_conv_bench.py [--batch 128] [--iters 10]
"""
import argparse
import collections
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_amd.models.resnet import resnet50  # noqa: E402
from distributed_pytorch_amd.ops import functional as Fn  # noqa: E402
from distributed_pytorch_amd.ops.layers import Conv2d  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def shapes(batch):
    m = resnet50(1000, "bf16").cuda()
    seen = collections.Counter()
    hooks = []
    for mod in m.modules():
        if isinstance(mod, Conv2d):
            def hook(mod, inp, out):
                x = inp[0]
                seen[(x.shape[0], x.shape[1], x.shape[2], mod.cin_pad, mod.cout, mod.k, mod.stride, mod.padding)] += 1
            hooks.append(mod.register_forward_hook(hook))
    with torch.no_grad():
        m(torch.zeros(batch, 224, 224, 3, device="cuda"))
    for h in hooks:
        h.remove()
    return seen


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    tot = collections.Counter()
    for (N, H, W, C, K, R, s, p), cnt in sorted(shapes(a.batch).items()):
        stem = R == 7  # the network input needs no gradient: weight gradient only
        x = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16).requires_grad_(not stem)
        w = (torch.randn(K, R, R, C, device="cuda") * 0.05).requires_grad_(True)
        z = Fn.conv2d_nhwc(x, w, s, p, "bf16")
        dz = torch.randn_like(z)
        ours_f = timeit(lambda: Fn.conv2d_nhwc(x, w, s, p, "bf16"), a.iters)
        ins = (w,) if stem else (x, w)
        ours_b = timeit(lambda: torch.autograd.grad(Fn.conv2d_nhwc(x, w, s, p, "bf16"), ins, dz), a.iters) - ours_f
        xt = x.detach().permute(0, 3, 1, 2).requires_grad_(not stem)  # channels_last view
        wt = w.detach().permute(0, 3, 1, 2).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt.requires_grad_(True)
        zt = F.conv2d(xt, wt, stride=s, padding=p)
        dzt = torch.randn_like(zt)
        th_f = timeit(lambda: F.conv2d(xt, wt, stride=s, padding=p), a.iters)
        ins_t = (wt,) if stem else (xt, wt)
        th_b = timeit(lambda: torch.autograd.grad(F.conv2d(xt, wt, stride=s, padding=p), ins_t, dzt),
                      a.iters) - th_f
        xw = x.detach()  # weight gradient alone (no data gradient requested)
        ours_w = timeit(lambda: torch.autograd.grad(Fn.conv2d_nhwc(xw, w, s, p, "bf16"), (w,), dz), a.iters) - ours_f
        row = {"shape": [N, H, W, C, K, R, s, p], "count": cnt, "ours_fwd": round(ours_f, 1),
               "ours_bwd": round(ours_b, 1), "ours_wgrad": round(ours_w, 1), "miopen_fwd": round(th_f, 1),
               "miopen_bwd": round(th_b, 1)}
        tot["ours"] += cnt * (ours_f + ours_b)
        tot["ours_wgrad"] += cnt * ours_w
        tot["miopen"] += cnt * (th_f + th_b)
        best_gemm = None
        if R == 1 and s == 1:
            M = N * H * W
            x2 = x.detach().view(M, C)
            w2 = w.detach().to(torch.bfloat16).view(K, C)
            dz2 = dz.view(M, K)
            g_f = timeit(lambda: x2 @ w2.t(), a.iters)
            g_b = timeit(lambda: (dz2 @ w2, dz2.t() @ x2), a.iters)
            row["gemm_fwd"], row["gemm_bwd"] = round(g_f, 1), round(g_b, 1)
            row["gemm_wgrad"] = round(timeit(lambda: dz2.t() @ x2, a.iters), 1)
            best_gemm = g_f + g_b
        tot["best"] += cnt * min(ours_f + ours_b, th_f + th_b, best_gemm or 1e18)
        print(json.dumps(row), flush=True)
    print(json.dumps({k: round(v / 1e3, 3) for k, v in tot.items()} | {"unit": "ms per step (convs only)"}),
          flush=True)


if __name__ == "__main__":
    main()
