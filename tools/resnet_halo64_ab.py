"""Isolated A/B of the 64-channel-chunk halo tiles (22 / 23, one bf16 plane) against the tuned plan of
every stride-1 3x3 conv call of ResNet-50 bf16 at batch 128 (tuning/generic_mi355x.json), as the
generic path issues them (bf16 NHWC in and out, split-K slabs reduced into bf16).

Prints one line per call and writes ``--out`` (JSON: key, current, best, all timings) and
``--cands`` (the faster plans in tools/adopt-style form {key: [tile, splits, pm, ms]}).

    python tools/resnet_halo64_ab.py [--out gpurun_out/resnet_halo64_ab.json]
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_pytorch_amd import _ext  # noqa: E402
from distributed_pytorch_amd.engine import halo_ok  # noqa: E402

GEOMS = [(56, 64), (28, 128), (14, 256), (7, 512)]  # stride-1 3x3 convs of the bottlenecks: (H = W, C = K)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--min-gain", type=float, default=0.03)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "resnet_halo64_ab.json"))
    ap.add_argument("--cands", default=os.path.join(ROOT, "gpurun_out", "resnet_halo64_cands.json"))
    a = ap.parse_args()
    K_ = _ext.require()
    table = json.load(open(os.path.join(ROOT, "distributed_pytorch_amd", "tuning", "generic_mi355x.json")))
    n = a.batch
    dev = "cuda"
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    rows, cands = [], {}
    for hw, c in GEOMS:
        x = (torch.randn(1, n, hw, hw, c, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn(1, c, 3, 3, c, device=dev) * 0.05).to(torch.bfloat16)
        out = torch.empty(n, hw, hw, c, device=dev, dtype=torch.bfloat16)
        for kind in ("fprop", "dgrad"):
            key = "|".join(str(v) for v in ("bf16", kind, n, hw, hw, c, c, 3, 3, 1, 1))
            t = table.get(key)
            if t is None:
                continue
            cur = (int(t[0]), int(t[1]), int(bool(t[2])))
            plans = [cur] + [(tile, s, 0) for tile in (22, 23) for s in (1, 2, 4)
                             if halo_ok(kind, tile, hw, c, c, 1) and c // 64 >= s]

            def run(p):
                tile, s, pm = p
                s = K_.x3_splits(9 * c, s)
                slab = torch.empty(s * n * hw * hw * c, device=dev) if s > 1 else None
                if kind == "fprop":
                    K_.conv_x3_fprop(x, w, out, slab, 1, 1, s, tile, True, pm, None)
                else:
                    K_.conv_x3_dgrad(x, w, out, slab, 1, 1, s, tile, True, pm, None)

            times = {p: [] for p in plans}
            for _ in range(a.rounds):
                for p in plans:
                    run(p)
                    ev0.record()
                    for _ in range(a.iters):
                        run(p)
                    ev1.record()
                    torch.cuda.synchronize()
                    times[p].append(ev0.elapsed_time(ev1) / a.iters * 1e3)
            med = {p: statistics.median(v) for p, v in times.items()}
            best = min(med, key=med.get)
            rows.append({"key": key, "current": list(cur), "current_us": med[cur], "best": list(best),
                         "best_us": med[best], "all": {f"{p[0]}/{p[1]}": round(v, 2) for p, v in med.items()}})
            if best != cur and med[best] < med[cur] * (1 - a.min_gain):
                cands[key] = [best[0], best[1], best[2], med[best] / 1e3]
            print(f"{key:40s} cur {cur} {med[cur]:7.2f} us  best {best} {med[best]:7.2f} us  {rows[-1]['all']}",
                  flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(rows, open(a.out, "w"), indent=1)
    json.dump(cands, open(a.cands, "w"), indent=1)


if __name__ == "__main__":
    main()
