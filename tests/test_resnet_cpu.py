"""ResNet (NHWC kernel layers) vs the stock-torch NCHW oracle, on the CPU path of the same
autograd functions: forward, backward, BN running statistics and state_dict interchange."""
import torch

from distributed_pytorch_amd.models.resnet import ResNet, ResNetRef, resnet50


def _pair(layers, classes=10, seed=0):
    """float64 on both sides: isolates the algorithm from fp32 rounding amplified by BN on a tiny
    batch (the GPU tests check fp32/bf16 numerics of the kernels themselves)."""
    torch.manual_seed(seed)
    ours = ResNet(layers, classes).double()
    ref = ResNetRef(layers, classes).double()
    ref.load_state_dict(ours.state_dict())
    return ours, ref


def test_state_dict_matches_torch_layout():
    m = resnet50()
    sd = m.state_dict()
    ref = ResNetRef([3, 4, 6, 3]).state_dict()
    assert list(sd.keys()) == list(ref.keys())
    for k in sd:
        assert sd[k].shape == ref[k].shape, k
    n = sum(p.numel() for p in ResNetRef([3, 4, 6, 3]).parameters())
    assert n == 25557032  # torchvision resnet50
    # round trip
    m2 = resnet50()
    m2.load_state_dict(sd)
    for (k, a), b in zip(m2.state_dict().items(), sd.values()):
        assert torch.equal(a, b), k


def test_forward_backward_matches_reference():
    ours, ref = _pair([1, 2, 1, 1])
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, 3, 48, 48, generator=g, dtype=torch.float64)
    t = torch.randint(0, 10, (4,), generator=g)
    lo = ours(x.permute(0, 2, 3, 1).contiguous())
    lr = ref(x)
    assert torch.allclose(lo, lr, rtol=1e-9, atol=1e-9), (lo - lr).abs().max()
    torch.nn.functional.cross_entropy(lo, t).backward()
    torch.nn.functional.cross_entropy(lr, t).backward()
    po = dict(ours.named_parameters())
    for name, p in ref.named_parameters():
        q = po[name].grad
        if q.dim() == 4:  # KRSC (padded) -> OIHW
            q = q[..., :p.shape[1]].permute(0, 3, 1, 2)
        err = (q - p.grad).abs().max() / p.grad.abs().max().clamp_min(1e-12)
        assert err < 1e-8, (name, float(err))
    so, sr = ours.state_dict(), ref.state_dict()
    for k in sr:
        if "running" in k or "num_batches" in k:
            assert torch.allclose(so[k].double(), sr[k].double(), rtol=1e-9, atol=1e-9), k


def test_eval_mode_uses_running_stats():
    ours, ref = _pair([1, 1, 1, 1])
    x = torch.randn(2, 3, 32, 32, dtype=torch.float64)
    ours(x.permute(0, 2, 3, 1).contiguous())  # one training step of stats
    ref(x)
    ours.eval()
    ref.eval()
    with torch.no_grad():
        assert torch.allclose(ours(x.permute(0, 2, 3, 1).contiguous()), ref(x), rtol=1e-9, atol=1e-9)


def test_ddp_arena_holds_gradient_of_a_weight_used_twice():
    """A conv weight / BN affine used twice in one forward: both uses' gradients must reach the
    arena slot the collectives and FlatSGD read (not just p.grad)."""
    import torch.nn as nn

    from distributed_pytorch_amd.ops.layers import BatchNorm2d, Conv2d
    from distributed_pytorch_amd.parallel.ddp import DistributedDataParallel

    class Twice(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv = Conv2d(8, 8, 3, 1, 1, impl="x3")
            self.bn = BatchNorm2d(8, act="relu")
            self.once = Conv2d(8, 8, 3, 1, 1, impl="x3")

        def forward(self, x):
            y = self.bn(self.conv(x))
            y = self.bn(self.conv(y))  # same weight, same BN affine, second use
            return self.once(y)

    torch.manual_seed(0)
    ref = Twice().double()
    m = Twice().double()
    m.load_state_dict(ref.state_dict())
    ddp = DistributedDataParallel(m, bucket_mb=0.01)
    x = torch.randn(2, 6, 6, 8, dtype=torch.float64)
    for it in range(2):  # the second iteration runs with the arena views already adopted
        ddp.zero_grad()
        ddp(x).square().sum().backward()
        ddp.finish()
        ref.zero_grad()
        ref(x).square().sum().backward()
        po = dict(m.named_parameters())
        for n, p in ref.named_parameters():
            i = next(j for j, q in enumerate(ddp._params) if q is po[n])
            arena = ddp._gflat.view(i, po[n])
            assert torch.allclose(arena, p.grad, rtol=1e-10, atol=1e-12), (it, n)
            assert torch.allclose(po[n].grad, p.grad, rtol=1e-10, atol=1e-12), (it, n)


def test_fused_head_loss_matches_reference():
    """model(x, target): GAP + Linear + softmax-CE in one node (ops/functional.HeadCE) == stock
    cross_entropy on the reference network, loss and every gradient (float64)."""
    ours, ref = _pair([1, 1, 1, 1])
    g = torch.Generator().manual_seed(7)
    x = torch.randn(3, 3, 40, 40, generator=g, dtype=torch.float64)
    t = torch.randint(0, 10, (3,), generator=g)
    lo = ours(x.permute(0, 2, 3, 1).contiguous(), t)
    lr = torch.nn.functional.cross_entropy(ref(x), t)
    assert torch.allclose(lo, lr, rtol=1e-10, atol=1e-12)
    (2.5 * lo).backward()
    (2.5 * lr).backward()
    po = dict(ours.named_parameters())
    for name, p in ref.named_parameters():
        q = po[name].grad
        if q.dim() == 4:
            q = q[..., :p.shape[1]].permute(0, 3, 1, 2)
        err = (q - p.grad).abs().max() / p.grad.abs().max().clamp_min(1e-12)
        assert err < 1e-8, (name, float(err))


def test_gradjoin_order_independent():
    from distributed_pytorch_amd.ops.functional import GradJoin

    a, b = torch.randn(5), torch.randn(5)
    for first, second in ((a, b), (b, a)):
        j = GradJoin(2)
        assert j.contribute(first.clone()) is None
        assert torch.allclose(j.contribute(second.clone()), a + b)
        assert j.left == 2 and j.buf is None  # reset for the next step
