"""Block-by-block forward activation and gradient error of the small x3 ResNet vs fp64 (and the
stock torch fp32 yardstick): where does the gradient error enter?"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_amd.models import resnet as R  # noqa: E402


def capture(model, blocks_attr, nhwc):
    acts, grads = {}, {}

    def mk(name):
        def fhook(mod, inp, out):
            o = out
            acts[name] = (o.permute(0, 3, 1, 2) if nhwc else o).detach().double().cpu()
            o.register_hook(lambda g: grads.__setitem__(name, (g.permute(0, 3, 1, 2) if nhwc else g).double().cpu()))
        return fhook

    for li in range(1, 5):
        for bi, b in enumerate(getattr(model, f"layer{li}")):
            b.register_forward_hook(mk(f"layer{li}.{bi}"))
    return acts, grads


def rel(a, b):
    return ((a - b).abs().max() / b.abs().max()).item()


def main():
    torch.manual_seed(0)
    base = R.ResNet([1, 2, 1, 1], 10, impl="x3")
    sd = base.state_dict()
    ref = R.ResNetRef([1, 2, 1, 1], 10).double()
    ref.load_state_dict(sd)
    r32 = R.ResNetRef([1, 2, 1, 1], 10)
    r32.load_state_dict(sd)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(8, 3, 64, 64, generator=g, dtype=torch.float64)
    t = torch.randint(0, 10, (8,), generator=g)
    a64, g64 = capture(ref, None, False)
    F.cross_entropy(ref(x), t).backward()
    a32, g32 = capture(r32, None, False)
    F.cross_entropy(r32(x.float()), t).backward()
    m = R.ResNet([1, 2, 1, 1], 10, impl="x3")
    m.load_state_dict(sd)
    m = m.cuda()
    ao, go = capture(m, None, True)
    m(x.permute(0, 2, 3, 1).float().contiguous().cuda(), t.cuda()).backward()
    torch.cuda.synchronize()
    print(f"{'block':10s} {'act ours':>10s} {'act t32':>10s} {'grad ours':>10s} {'grad t32':>10s}")
    for k in a64:
        print(f"{k:10s} {rel(ao[k], a64[k]):10.2e} {rel(a32[k], a64[k]):10.2e} {rel(go[k], g64[k]):10.2e} "
              f"{rel(g32[k], g64[k]):10.2e}")


if __name__ == "__main__":
    main()
