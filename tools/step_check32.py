"""test_ops_gpu.py::test_engine_step_matches_torch at N=32: per-tensor error of the engine (fp32 /
x3 / h2) and of torch fp32 vs fp64, and the closest ReLU / max-pool decision margins of the fp64
forward per layer (a margin below the step's rounding means a routing flip is possible)."""
import sys, os
import torch
import torch.nn as nn
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_pytorch_amd.engine import VGGEngine  # noqa: E402
from distributed_pytorch_amd.models import VGG11  # noqa: E402

torch.manual_seed(1)
m = VGG11().double()
N = 32
x = torch.randn(N, 3, 32, 32, dtype=torch.float64)
t = torch.randint(0, 10, (N,))
m32 = VGG11()
m32.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in m.state_dict().items()})
acts = []
for mod in m.modules():
    if isinstance(mod, nn.BatchNorm2d):
        mod.register_forward_hook(lambda mm, i, o: acts.append(o.detach()))
F.cross_entropy(m(x), t).backward()
F.cross_entropy(m32(x.float()), t).backward()
for li, y in enumerate(acts):  # BN outputs: ReLU margin = min |y|; pool margin = top-2 gap of relu(y)
    r = torch.relu(y)
    n, c, h, w = r.shape
    win = r.reshape(n, c, h // 2, 2, w // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(n, c, h // 2, w // 2, 4)
    top = win.sort(-1, descending=True).values
    gap = (top[..., 0] - top[..., 1])[top[..., 0] > 0]
    print(f"layer {li}: min |bn out| {y.abs().min().item():.2e}  min pool gap {gap.min().item():.2e}")
ref = {n: p.grad for n, p in m.named_parameters()}
t32 = {n: p.grad.double() for n, p in m32.named_parameters()}
for impl in ("fp32", "x3", "h2"):
    e = VGGEngine("VGG11", "cuda", max_batch=N, impl=impl)
    e.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in m.state_dict().items()})
    x4 = torch.zeros(N, 32, 32, 4)
    x4[..., :3] = x.float().permute(0, 2, 3, 1)
    e.forward_backward(x4.cuda(), t.cuda())
    torch.cuda.synchronize()
    worst = []
    for n, g in ref.items():
        if g.abs().max() < 1e-6:
            continue
        gd = e._to_torch_layout(n, e.grads[n]).cpu().double()
        s = g.abs().max().item()
        worst.append(((gd - g).abs().max().item() / s, (t32[n] - g).abs().max().item() / s, n))
    worst.sort(reverse=True)
    print(impl, [(f"{a:.1e}", f"{b:.1e}", n) for a, b, n in worst[:4]])
