"""Inside one ResNet bottleneck (layer3.0 of a small x3 ResNet): forward / gradient error of every
module output vs fp64, to find where a parameter-gradient error enters."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_amd.models import resnet as R  # noqa: E402


def hook_all(block, nhwc, store):
    names = ["conv1", "bn1", "conv2", "bn2", "conv3", "bn3", "downsample.0", "downsample.1"]
    mods = dict(block.named_modules())
    for n in names:
        m = mods[n]

        def fh(mod, inp, out, n=n):
            o = out
            store["act"][n] = (o.permute(0, 3, 1, 2) if nhwc else o).detach().double().cpu()
            o.register_hook(lambda g: store["grad"].__setitem__(n, (g.permute(0, 3, 1, 2) if nhwc else g).double().cpu()))
        m.register_forward_hook(fh)


def rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def main():
    torch.manual_seed(0)
    base = R.ResNet([1, 2, 1, 1], 10, impl="x3")
    sd = base.state_dict()
    ref = R.ResNetRef([1, 2, 1, 1], 10).double()
    ref.load_state_dict(sd)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(8, 3, 64, 64, generator=g, dtype=torch.float64)
    t = torch.randint(0, 10, (8,), generator=g)
    s64 = {"act": {}, "grad": {}}
    hook_all(ref.layer3[0], False, s64)
    F.cross_entropy(ref(x), t).backward()
    m = R.ResNet([1, 2, 1, 1], 10, impl="x3")
    m.load_state_dict(sd)
    m = m.cuda()
    so = {"act": {}, "grad": {}}
    hook_all(m.layer3[0], True, so)
    m(x.permute(0, 2, 3, 1).float().contiguous().cuda(), t.cuda()).backward()
    torch.cuda.synchronize()
    for n in s64["act"]:
        print(f"{n:14s} act {rel(so['act'][n], s64['act'][n]):9.2e}  grad {rel(so['grad'][n], s64['grad'][n]):9.2e}"
              f"  |grad| {s64['grad'][n].abs().max().item():9.2e}")
    po, pr = dict(m.layer3[0].named_parameters()), dict(ref.layer3[0].named_parameters())
    for n, p in pr.items():
        q = po[n].grad
        if q.dim() == 4:
            q = q[..., :p.shape[1]].permute(0, 3, 1, 2)
        print(f"param {n:22s} {rel(q, p.grad):9.2e}")


if __name__ == "__main__":
    main()
