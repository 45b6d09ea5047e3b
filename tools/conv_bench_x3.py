"""Per-layer timing of the bf16-plane conv kernels (np=3: fp32-grade via bf16x6; np=1: bf16) on
the VGG-11 shapes at batch 256.

    python tools/conv_bench_x3.py [--np 3] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_amd import _ext  # noqa: E402

VGG11 = [(16, 64, 128), (8, 128, 256), (8, 256, 256), (4, 256, 512), (4, 512, 512), (2, 512, 512)]


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
    ap.add_argument("--np", type=int, default=3)
    a = ap.parse_args()
    C = _ext.require()
    N, NP = a.batch, a.np
    tot = 0.0
    for (H, Cin, K) in VGG11:
        x3 = torch.randn(NP, N, H, H, Cin, device="cuda").bfloat16()
        w3 = (torch.randn(NP, K, 3, 3, Cin, device="cuda") * 0.05).bfloat16()
        dz3 = torch.randn(NP, N, H, H, K, device="cuda").bfloat16()
        z = torch.empty(N, H, H, K, device="cuda")
        dx = torch.empty(N, H, H, Cin, device="cuda")
        dw = torch.empty(K, 3, 3, Cin, device="cuda")
        M = N * H * H
        flops = 2.0 * M * K * 9 * Cin
        slab = torch.empty(128 * max(M * max(K, Cin), K * 9 * Cin), device="cuda")
        best = {}
        for kind in ("fprop", "dgrad", "wgrad"):
            res = []
            for tile, pm in [(t, p) for t in (0, 1, 2, 3, 4, 5, 6, 7) for p in (False, True)]:
                for splits in (1, 2, 4, 8, 16, 32, 64, 128):
                    if kind != "wgrad" and splits > 16:
                        continue
                    if kind == "fprop":
                        fn = lambda: C.conv_x3_fprop(x3, w3, z, slab, 1, 1, splits, tile, False, pm)
                    elif kind == "dgrad":
                        fn = lambda: C.conv_x3_dgrad(dz3, w3, dx, slab, 1, 1, splits, tile, False, pm)
                    else:
                        fn = lambda: C.conv_x3_wgrad(x3, dz3, dw, slab, 1, 1, splits, tile, pm)
                    res.append((timeit(fn, a.iters), tile, splits, pm))
            res.sort()
            best[kind] = res[0]
        tot += sum(b[0] for b in best.values())
        print(json.dumps({"H": H, "Cin": Cin, "K": K, "np": NP,
                          "best": {k: {"ms": round(v[0], 4), "tile": v[1], "splits": v[2], "posmajor": v[3],
                                       "tflops_eq": round(flops / v[0] / 1e9, 1)} for k, v in best.items()}}),
              flush=True)
    print(json.dumps({"total_ms_excl_layer0": round(tot, 3), "np": NP}))


if __name__ == "__main__":
    main()
