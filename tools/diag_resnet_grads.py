"""Per-tensor gradient error of the small x3 ResNet vs fp64, for the head / GradJoin variants and
stock torch fp32 (yardstick).  Diagnostic for tests/test_layers_gpu.py."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_amd.models import resnet as R  # noqa: E402
from distributed_pytorch_amd.ops import functional as Fn  # noqa: E402


def errs(model_grads, ref):
    out = {}
    for n, p in ref.named_parameters():
        q = model_grads[n]
        if q.dim() == 4 and q.shape != p.shape:
            q = q[..., :p.shape[1]].permute(0, 3, 1, 2)
        out[n] = ((q.double().cpu() - p.grad).abs().max() / p.grad.abs().max()).item()
    return out


def main():
    torch.manual_seed(0)
    base = R.ResNet([1, 2, 1, 1], 10, impl="x3")
    sd = base.state_dict()
    ref = R.ResNetRef([1, 2, 1, 1], 10).double()
    ref.load_state_dict(sd)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(8, 3, 64, 64, generator=g, dtype=torch.float64)
    t = torch.randint(0, 10, (8,), generator=g)
    F.cross_entropy(ref(x), t).backward()
    r32 = R.ResNetRef([1, 2, 1, 1], 10)
    r32.load_state_dict(sd)
    F.cross_entropy(r32(x.float()), t).backward()
    res = {"torch_fp32": errs({n: p.grad for n, p in r32.named_parameters()}, ref)}
    xin = x.permute(0, 2, 3, 1).float().contiguous().cuda()
    for variant in ("fused_loss", "logits_head", "no_join"):
        m = R.ResNet([1, 2, 1, 1], 10, impl="x3")
        m.load_state_dict(sd)
        m = m.cuda()
        if variant == "no_join":
            for mod in m.modules():
                if isinstance(mod, R.Bottleneck):
                    mod._join = None
                    mod.forward = (lambda self: (lambda xx: self.bn3(self.conv3(self.bn2(self.conv2(self.bn1(
                        self.conv1(xx))))), self.downsample[1](self.downsample[0](xx)) if self.downsample is not None
                        else xx)))(mod)
        if variant == "fused_loss":
            m(xin, t.cuda()).backward()
        else:
            F.cross_entropy(m(xin), t.cuda()).backward()
        torch.cuda.synchronize()
        res[variant] = errs({n: p.grad for n, p in m.named_parameters()}, ref)
    names = list(res["torch_fp32"])
    print(f"{'param':34s} " + " ".join(f"{k:>12s}" for k in res))
    for n in names:
        print(f"{n:34s} " + " ".join(f"{res[k][n]:12.2e}" for k in res))


if __name__ == "__main__":
    main()
