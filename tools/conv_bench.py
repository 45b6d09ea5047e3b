"""Per-layer timing of the HIP conv kernels (fprop / dgrad / wgrad) on the VGG-11 shapes at
batch 256, against MIOpen (torch.nn.functional.conv2d fp32, channels_last) on the same GPU.

    python tools/conv_bench.py [--iters 20]
"""
import argparse
import json

import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_amd import _ext  # noqa: E402

# (H, C_in, K)  3x3 s1 p1, batch 256 — SURVEY §2.3 implicit-GEMM dims
VGG11 = [(32, 4, 64), (16, 64, 128), (8, 128, 256), (8, 256, 256), (4, 256, 512), (4, 512, 512), (2, 512, 512),
         (2, 512, 512)]


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--configs", default="")
    a = ap.parse_args()
    C = _ext.require()
    N = a.batch
    tot = {"ours": 0.0, "miopen": 0.0}
    for (H, Cin, K) in VGG11:
        x = torch.randn(N, H, H, Cin, device="cuda")
        w = torch.randn(K, 3, 3, Cin, device="cuda") * 0.05
        z = torch.empty(N, H, H, K, device="cuda")
        dz = torch.randn(N, H, H, K, device="cuda")
        wf = torch.empty(Cin, 3, 3, K, device="cuda")
        dx = torch.empty(N, H, H, Cin, device="cuda")
        dw = torch.empty(K, 3, 3, Cin, device="cuda")
        M = N * H * H
        flops = 2.0 * M * K * 9 * Cin
        best = {}
        for kind in ("fprop", "dgrad", "wgrad"):
            res = []
            for tile, pm in ((0, False), (1, False), (0, True), (1, True)):
                for splits in (1, 2, 4, 8, 16, 32, 64, 128):
                    if kind == "fprop":
                        need = splits * M * K
                        slab = torch.empty(need, device="cuda") if splits > 1 else None
                        fn = lambda: C.conv_fprop(x, w, z, slab, 1, 1, splits, tile, False, True, pm)
                    elif kind == "dgrad":
                        need = splits * M * Cin
                        slab = torch.empty(need, device="cuda") if splits > 1 else None
                        fn = lambda: C.conv_fprop(dz, w, dx, slab, 1, 1, splits, tile, True, True, pm)
                    else:
                        need = splits * K * 9 * Cin
                        slab = torch.empty(need, device="cuda") if splits > 1 else None
                        fn = lambda: C.conv_wgrad(x, dz, dw, slab, 1, 1, splits, tile, pm)
                    if kind != "wgrad" and splits > 16:
                        continue
                    ms = timeit(fn, a.iters)
                    res.append((ms, tile, splits, pm))
            res.sort()
            best[kind] = res[0]
        # MIOpen reference (NCHW-logical, channels_last memory)
        xc = x.permute(0, 3, 1, 2)
        wc = w.permute(0, 3, 1, 2).contiguous().to(memory_format=torch.channels_last)
        xg = xc.detach().requires_grad_(True)
        wg = wc.detach().requires_grad_(True)
        dzc = dz.permute(0, 3, 1, 2)
        mi_f = timeit(lambda: F.conv2d(xc, wc, padding=1), a.iters)
        yy = F.conv2d(xg, wg, padding=1)
        mi_b = timeit(lambda: torch.autograd.grad(yy, (xg, wg), dzc, retain_graph=True), a.iters)
        ours = sum(b[0] for b in best.values())
        tot["ours"] += ours
        tot["miopen"] += mi_f + mi_b
        print(json.dumps({"H": H, "Cin": Cin, "K": K, "gflop": flops / 1e9,
                          "best": {k: {"ms": round(v[0], 4), "tile": v[1], "splits": v[2], "posmajor": v[3],
                                       "tflops": round(flops / v[0] / 1e9, 1)} for k, v in best.items()},
                          "miopen_fwd_ms": round(mi_f, 4), "miopen_bwd_ms": round(mi_b, 4)}), flush=True)
    print(json.dumps({"total_ms": {k: round(v, 3) for k, v in tot.items()}}))


if __name__ == "__main__":
    main()
