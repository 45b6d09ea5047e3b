"""Isolated timing: the 2x2 VGG layers (512 -> 512, 3x3, pad 1, batch 256) as 3x3 convs against
the same layers written as one dense GEMM.  On a 2x2 image every output pixel sees the whole input
through 4 of the 9 taps, so z[n,(p,co)] = sum_(q,ci) Wd[(p,co),(q,ci)] x[n,(q,ci)] with
Wd[(p,co),(q,ci)] = W[co, ci, q-p+(1,1)]: a 1x1 conv on a 1x1 image with 2048 channels.

    python tools/micro_dense2x2.py [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_amd import _ext  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def sweep(C, fns, iters, max_split):
    res = []
    for tile in range(0, 22):
        for pm in (False, True):
            for splits in (1, 2, 4, 8, 16, 32):
                if splits > max_split:
                    continue
                try:
                    ms = timeit(lambda: fns(tile, splits, pm), iters)
                except RuntimeError:
                    continue
                res.append((ms, tile, splits, pm))
    res.sort()
    return res[:4]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    C = _ext.require()
    N, NP = 256, 3
    slab = torch.empty(32 * 2048 * 2048, device="cuda")
    out = {}
    # 3x3 form on the 2x2 image (current engine path)
    x3 = torch.randn(NP, N, 2, 2, 512, device="cuda").bfloat16()
    w3 = (torch.randn(NP, 512, 3, 3, 512, device="cuda") * 0.05).bfloat16()
    dz3 = torch.randn(NP, N, 2, 2, 512, device="cuda").bfloat16()
    z = torch.empty(N, 2, 2, 512, device="cuda")
    dw = torch.empty(512, 3, 3, 512, device="cuda")
    out["conv3x3"] = {
        "fprop": sweep(C, lambda t, s, p: C.conv_x3_fprop(x3, w3, z, slab, 1, 1, s, t, False, p), a.iters, 16),
        "dgrad": sweep(C, lambda t, s, p: C.conv_x3_dgrad(dz3, w3, z, slab, 1, 1, s, t, False, p), a.iters, 16),
        "wgrad": sweep(C, lambda t, s, p: C.conv_x3_wgrad(x3, dz3, dw, slab, 1, 1, s, t, p), a.iters, 32),
    }
    print(json.dumps({"conv3x3": out["conv3x3"]}), flush=True)
    # dense form: 1x1 conv on a 1x1 image, 2048 -> 2048 channels
    xd = x3.view(NP, N, 1, 1, 2048)
    wd = (torch.randn(NP, 2048, 1, 1, 2048, device="cuda") * 0.05).bfloat16()
    dzd = dz3.view(NP, N, 1, 1, 2048)
    zd = torch.empty(N, 1, 1, 2048, device="cuda")
    dwd = torch.empty(2048, 1, 1, 2048, device="cuda")
    out["dense"] = {
        "fprop": sweep(C, lambda t, s, p: C.conv_x3_fprop(xd, wd, zd, slab, 1, 0, s, t, False, p), a.iters, 16),
        "dgrad": sweep(C, lambda t, s, p: C.conv_x3_dgrad(dzd, wd, zd, slab, 1, 0, s, t, False, p), a.iters, 16),
        "wgrad": sweep(C, lambda t, s, p: C.conv_x3_wgrad(xd, dzd, dwd, slab, 1, 0, s, t, p), a.iters, 32),
    }
    print(json.dumps({"dense": out["dense"]}), flush=True)


if __name__ == "__main__":
    main()
