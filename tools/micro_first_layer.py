"""Isolated timings of the first-layer kernels at batch 256 (fused vs the generic path).

    python tools/micro_first_layer.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_amd.engine import VGGEngine  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    N = 256
    e = VGGEngine("VGG11", "cuda", max_batch=N, impl="x3")
    e.init_parameters(seed=1)
    x = torch.zeros(N, 32, 32, 4, device="cuda")
    x[..., :3] = torch.randn(N, 32, 32, 3, device="cuda")
    t = torch.randint(0, 10, (N,), device="cuda")
    e.forward_backward(x, t)
    K, P, G = e.K, e.params, e.grads
    l = e.spec.convs[0]
    st = e.stats[0]
    w = P[f"{l.conv_key}.weight"]
    bnargs = (P[f"{l.bn_key}.weight"], P[f"{l.bn_key}.bias"], P[f"{l.conv_key}.bias"],
              e.buffers[f"{l.bn_key}.running_mean"], e.buffers[f"{l.bn_key}.running_var"], e.nbt[0:1], st["mean"],
              st["invstd"], st["scale"], st["shift"], 0.1, 1e-5)
    z = e.z[0]
    res = {}
    res["conv0_fwd+stats+finalize"] = timeit(lambda: K.conv0_fwd(x, w, z, e.part0, *bnargs))
    res["conv0_fwd (eval, conv only)"] = timeit(lambda: K.conv0_fwd(x, w, z))

    def generic_fwd():
        K.pad_split8(x, e.x0p)
        ns = e._conv_fwd(0, x, N, reduce=False)
        K.bn_fwd_stats(e.slab if ns > 1 else z, ns, z, e.part, *bnargs)
    res["pad_split8+x3 conv+bn_stats+finalize"] = timeit(generic_fwd)
    g = e.g[0]
    bw = (st["scale"], st["shift"], st["mean"], st["invstd"], P[f"{l.bn_key}.weight"], e.part, e.coef,
          G[f"{l.bn_key}.weight"], G[f"{l.bn_key}.bias"], G[f"{l.conv_key}.bias"])
    res["bn_bwd_wgrad0 (fused)"] = timeit(lambda: K.bn_bwd_wgrad0(g, 1, g, z, *bw, x, e.wpart,
                                                                  G[f"{l.conv_key}.weight"]))

    def generic_bwd():
        K.pad_split8(x, e.x0p)
        K.bn_bwd(g, 1, g, z, *bw, e.dz3[0], True)
        e._conv_wgrad(0, x, N)
    res["bn_bwd + x3 wgrad"] = timeit(generic_bwd)
    for k, v in res.items():
        print(f"{v:8.1f} us  {k}")


if __name__ == "__main__":
    main()
