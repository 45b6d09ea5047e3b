"""Isolated A/B of the 64-channel-chunk halo tiles (22 = 256x128/64, 23 = 256x64/64) against the
current plan of every halo-tiled conv call of the VGG-11 h2 step (batch 256).

For each fprop / dgrad call whose table plan is a halo tile, times the current plan and tiles 22 /
23 at every split count that divides the chunks, ``--iters`` launches per measurement, ``--rounds``
interleaved rounds (median).  Prints one line per call and writes JSON to ``--out``.

    python tools/halo64_ab.py [--out gpurun_out/halo64_ab.json]
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_pytorch_amd.engine import VGGEngine, conv_key, halo_ok  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--impl", default="h2")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "halo64_ab.json"))
    ap.add_argument("--all", action="store_true", help="also calls whose current plan is not a halo tile")
    ap.add_argument("--only", default="", help="comma-separated conv_key substrings")
    a = ap.parse_args()
    n = a.batch
    e = VGGEngine("VGG11", "cuda", max_batch=n, impl=a.impl)
    x = torch.randn(n, 32, 32, 4, device="cuda")
    x[..., 3] = 0
    e.x0.copy_(x)
    t = torch.randint(0, 10, (n,), device="cuda")
    e.forward_backward(e.x0, t)
    torch.cuda.synchronize()
    np_ = {"x3": 3, "h2": 2}.get(a.impl, 1)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    rows = []
    for i, l in enumerate(e.spec.convs):
        for kind in ("fprop", "dgrad"):
            if i == 0:
                continue
            impl = e._layer_impl(i)
            key = (impl, kind, n, i)
            if a.only and not any(o in conv_key(impl, kind, n, l.hw, l.cin_pad, l.cout) for o in a.only.split(",")):
                continue
            cur = e.conv_config(i, kind, n)
            cred, cout = (l.cin_pad, l.cout) if kind == "fprop" else (l.cout, l.cin_pad)
            if not (16 <= cur[0] <= 23 or (a.all and halo_ok(kind, 22, l.hw, cred, cout, np_))):
                continue
            cands = [cur]
            for tile in (22, 23):
                if not halo_ok(kind, tile, l.hw, cred, cout, np_):
                    continue
                for s in (1, 2, 4, 8):
                    es = e.K.x3_splits(9 * cred, s)
                    c = (tile, es, 0)
                    if c not in cands and (cred // 64) >= s:
                        cands.append(c)
            fn = {"fprop": lambda: e._conv_fwd(i, e.x0[:n], n, reduce=False),
                  "dgrad": lambda: e._conv_dgrad(i, n)}[kind]
            times = {c: [] for c in cands}
            for _ in range(a.rounds):
                for c in cands:
                    e._cfg_cache[key] = c
                    e._ensure_slab(e._slab_need(i, kind, n))
                    fn()
                    ev0.record()
                    for _ in range(a.iters):
                        fn()
                    ev1.record()
                    torch.cuda.synchronize()
                    times[c].append(ev0.elapsed_time(ev1) / a.iters * 1e3)
            e._cfg_cache[key] = cur
            med = {c: statistics.median(v) for c, v in times.items()}
            best = min(med, key=med.get)
            ck = conv_key(impl, kind, n, l.hw, l.cin_pad, l.cout)
            row = {"key": ck, "layer": i, "current": list(cur), "current_us": med[cur],
                   "best": list(best), "best_us": med[best],
                   "all": {f"{c[0]}/{c[1]}": round(v, 2) for c, v in med.items()}}
            rows.append(row)
            print(f"{ck:28s} L{i} cur {cur} {med[cur]:7.2f} us  best {best} {med[best]:7.2f} us  "
                  f"{row['all']}", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
