"""EXPERIMENT: how much of a halo conv's time is operand staging?  Times the VGG-11 x3 forward halo
convs (tile 17, the engine's split counts) with parts of the staging switched off through
DPA_HALO_DBG (bit 0 B stores, 1 B loads, 2 A stores, 3 A loads; outputs are garbage then).  An upper
bound on what any staging change (direct-to-LDS loads included) can save.

    python tools/halo_staging_bound.py [--iters 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_amd import _ext  # noqa: E402

# (H, C_in, K, splits) of layers 1-5 at batch 256 (engine tuning table, tile 17)
LAYERS = [(16, 64, 128, 1), (8, 128, 256, 2), (8, 256, 256, 2), (4, 256, 512, 4), (4, 512, 512, 4)]


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
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--dgrad", action="store_true")
    a = ap.parse_args()
    K_ = _ext.require()
    N = a.batch
    for (H, C, K, s) in LAYERS:
        wp = (torch.randn(3, K, 3, 3, C, device="cuda") * 0.05).to(torch.bfloat16)
        if a.dgrad:  # dx [N,H,W,C] from dz [N,H,W,K] and the forward weights
            src = torch.randn(3, N, H, H, K, device="cuda").to(torch.bfloat16)
            out = torch.empty(N, H, H, C, device="cuda")
            slab = torch.empty(s * N * H * H * C, device="cuda") if s > 1 else None
            fn = lambda: K_.conv_x3_dgrad(src, wp, out, slab, 1, 1, s, 17, True, 0, None)
        else:
            src = torch.randn(3, N, H, H, C, device="cuda").to(torch.bfloat16)
            out = torch.empty(N, H, H, K, device="cuda")
            slab = torch.empty(s * N * H * H * K, device="cuda") if s > 1 else None
            fn = lambda: K_.conv_x3_fprop(src, wp, out, slab, 1, 1, s, 17, True, 0, None)
        row = {"kind": "dgrad" if a.dgrad else "fprop", "H": H, "C": C, "K": K, "splits": s}
        for dbg in (0, 1, 3, 4, 12, 15):
            os.environ["DPA_HALO_DBG"] = str(dbg)
            row[f"dbg{dbg}_us"] = round(timeit(fn, a.iters), 2)
        os.environ["DPA_HALO_DBG"] = "0"
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
