"""Where does the step's error first exceed stock torch fp32's?  At the trained state of
tests/test_parity256_gpu.py, compare every layer's conv output z, BN batch mean / invstd and the
backward's z-gradient-side quantities of the engine (fp32 / x3 / h2) and of torch fp32 (CPU) against
fp64 autograd of the same step.

    python tools/fwd_precision.py [--impls fp32,x3,h2] [--state trained|init]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _taps(model, x, t):
    """conv outputs (NCHW, with bias), BN batch mean / var of them, and the gradients wrt each conv
    output, from one forward + backward of ``model`` on (x, t)."""
    convs = [m for m in model.modules() if isinstance(m, nn.Conv2d)]
    outs = []

    def hook(m, i, o):
        o.retain_grad()
        outs.append(o)

    hs = [c.register_forward_hook(hook) for c in convs]
    loss = F.cross_entropy(model(x), t)
    loss.backward()
    for h in hs:
        h.remove()
    res = []
    for c, o in zip(convs, outs):
        od = o.detach().double()
        mean = od.mean((0, 2, 3))
        var = od.var((0, 2, 3), unbiased=False)
        res.append({"z": (od - c.bias.detach().double().view(1, -1, 1, 1)), "mean": mean - c.bias.detach().double(),
                    "invstd": torch.rsqrt(var + 1e-5), "dz": o.grad.detach().double()})
    return res


def rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impls", default="fp32,x3,h2")
    ap.add_argument("--state", default="trained")
    ap.add_argument("--out", default="gpurun_out/fwd_precision.json")
    a = ap.parse_args()
    import test_parity256_gpu as P
    from distributed_pytorch_amd.engine import VGGEngine
    from distributed_pytorch_amd.models import VGG11

    sd = P._trained_state() if a.state == "trained" else None
    ref = P._reference(sd, data_seed=512 if sd is not None else 256)
    m64 = VGG11().double()
    m64.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in ref["sd0"].items()})
    r64 = _taps(m64, ref["x"], ref["t"])
    m32 = VGG11()
    m32.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in ref["sd0"].items()})
    r32 = _taps(m32, ref["x"].float(), ref["t"])
    rows = {"torch_fp32": [], **{i: [] for i in a.impls.split(",")}}
    for i, l in enumerate(r64):
        q = r32[i]
        rows["torch_fp32"].append({"z": rel(q["z"], l["z"]), "mean_abs_over_std": float(((q["mean"] - l["mean"]).abs() * l["invstd"]).max()),
                                   "invstd": rel(q["invstd"], l["invstd"]), "dz": rel(q["dz"], l["dz"]),
                                   "absmean_over_std": float((l["mean"].abs() * l["invstd"]).max())})
    for impl in a.impls.split(","):
        e = VGGEngine("VGG11", "cuda", max_batch=P.N, impl=impl)
        e.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in ref["sd0"].items()})
        x4 = torch.zeros(P.N, 32, 32, 4)
        x4[..., :3] = ref["x"].float().permute(0, 2, 3, 1)
        e.forward_backward(x4.cuda(), ref["t"].cuda())
        torch.cuda.synchronize()
        for i, l in enumerate(r64):
            z = e.z[i].cpu().permute(0, 3, 1, 2)
            st = e.stats[i]
            rows[impl].append({"z": rel(z, l["z"]), "mean_abs_over_std": float(((st["mean"].cpu().double() - l["mean"]).abs() * l["invstd"]).max()),
                               "invstd": rel(st["invstd"].cpu(), l["invstd"])})
        del e
    print(f"{'layer':>5s} {'|mu|/sd':>8s} | " + " | ".join(f"{k:^30s}" for k in rows))
    print(f"{'':>5s} {'':>8s} | " + " | ".join(f"{'z':>9s} {'dmu/sd':>9s} {'invstd':>9s}" for _ in rows))
    for i in range(len(r64)):
        print(f"{i:5d} {rows['torch_fp32'][i]['absmean_over_std']:8.1f} | " + " | ".join(
            f"{rows[k][i]['z']:9.2e} {rows[k][i]['mean_abs_over_std']:9.2e} {rows[k][i]['invstd']:9.2e}" for k in rows))
    print("torch fp32 dz rel err per layer:", [f"{r['dz']:.2e}" for r in rows["torch_fp32"]])
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
