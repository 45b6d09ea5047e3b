"""Layer 0 of VGG-11 on its fused kernels (first_layer.hip conv0_fwd with the BN statistics in its
epilogue, bn_apply with the 2x2 max-pool, bn.hip bn_bwd_wgrad0: the BN backward apply fused with
the weight gradient) against torch autograd in fp64 — conv2d(3->64, 3x3, pad 1) ->
BatchNorm2d(train) -> ReLU -> MaxPool2d(2, 2), /root/reference/model.py:16-25.

Operands sit on coarse binary grids (x in quarters, w in eighths), so every conv output is exact
in fp32 and fp64 alike; beta puts each channel's ReLU threshold half-way between two output levels.
fp32 and fp64 then make the same 2x2 max-pool and ReLU decisions, and the comparison measures
arithmetic error only.  Windows whose maximum is an exact tie get a zero upstream gradient: torch's
own CPU kernels route a tie to different pixels on different machines.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

EPS, MOM = 1e-5, 0.1


def _C():
    from distributed_pytorch_amd import _ext

    return _ext.require()


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _case(N, CP, seed):
    g = torch.Generator().manual_seed(seed)
    x3 = torch.randint(-4, 5, (N, 3, 32, 32), generator=g).double() / 4
    w = torch.randint(-4, 5, (64, 3, 3, 3), generator=g).double() / 8  # OIHW
    z = F.conv2d(x3, w, padding=1)  # exact: multiples of 1/32
    gamma = torch.rand(64, generator=g, dtype=torch.float64) + 0.5
    bias = torch.randn(64, generator=g, dtype=torch.float64)
    zz = z.permute(0, 2, 3, 1).reshape(-1, 64)
    mu, var = zz.mean(0), zz.var(0, unbiased=False)
    thr = (torch.round(mu * 32) + torch.randint(-8, 9, (64,), generator=g).double() + 0.5) / 32  # between levels
    beta = -gamma * (thr - mu) * torch.rsqrt(var + EPS)
    rm, rv = torch.randn(64, generator=g, dtype=torch.float64), torch.rand(64, generator=g, dtype=torch.float64) + 0.5
    gout = torch.randn(N, 64, 16, 16, generator=g, dtype=torch.float64)
    # exact ties at a window's (positive) maximum are common on a grid; which tied pixel receives the
    # gradient is torch's choice and differs between its CPU kernels (vector widths), so those
    # windows carry no gradient and every valid routing gives the same result
    ypre = F.relu(F.batch_norm(z + bias.view(1, -1, 1, 1), None, None, gamma, beta, training=True, eps=EPS))
    win = ypre.reshape(N, 64, 16, 2, 16, 2).permute(0, 1, 2, 4, 3, 5).reshape(N, 64, 16, 16, 4)
    top = win.sort(-1, descending=True).values
    gout[(top[..., 0] == top[..., 1]) & (top[..., 0] > 0)] = 0.0
    # fp64 oracle (bias folded in as the kernels do: z excludes it)
    xx = x3.clone().requires_grad_(True)
    ww = w.clone().requires_grad_(True)
    bb = bias.clone().requires_grad_(True)
    gm, bt = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    rm_, rv_ = rm.clone(), rv.clone()
    y = F.max_pool2d(F.relu(F.batch_norm(F.conv2d(xx, ww, bb, padding=1), rm_, rv_, gm, bt, training=True,
                                         momentum=MOM, eps=EPS)), 2, 2)
    y.backward(gout)
    ref = dict(a=y.detach().permute(0, 2, 3, 1), rm=rm_, rv=rv_, mean=mu, invstd=torch.rsqrt(var + EPS),
               dw=ww.grad, dgamma=gm.grad, dbeta=bt.grad, dbias=bb.grad)
    x4 = torch.zeros(N, 32, 32, 4)
    x4[..., :3] = x3.permute(0, 2, 3, 1).float()
    wk = torch.zeros(64, 3, 3, CP)
    wk[..., :3] = w.permute(0, 2, 3, 1).float()  # KRSC, padded channels zero
    ops = dict(x=x4.cuda(), w=wk.cuda(), gamma=gamma.float().cuda(), beta=beta.float().cuda(),
               bias=bias.float().cuda(), rm=rm.float().cuda(), rv=rv.float().cuda(),
               gout=gout.permute(0, 2, 3, 1).float().contiguous().cuda())
    return ops, ref


@pytest.mark.parametrize("N,CP", [(256, 8), (16, 4), (2, 8)])
def test_layer0_fused_forward_and_backward(N, CP):
    C = _C()
    ops, ref = _case(N, CP, 10 + N)
    dev = "cuda"
    part = torch.zeros(C.conv0_part_floats(N), device=dev)
    mean, invstd, scale, shift = (torch.zeros(64, device=dev) for _ in range(4))
    rm, rv, nbt = ops["rm"].clone(), ops["rv"].clone(), torch.zeros(1, dtype=torch.int64, device=dev)
    z = torch.empty(N, 32, 32, 64, device=dev)
    C.conv0_fwd(ops["x"], ops["w"], z, part, ops["gamma"], ops["beta"], ops["bias"], rm, rv, nbt, mean, invstd, scale,
                shift, MOM, EPS)
    planes = torch.empty(3, N, 16, 16, 64, device=dev, dtype=torch.bfloat16)
    C.bn_apply(z, planes, scale, shift, True)
    a32 = torch.empty(N, 16, 16, 64, device=dev)
    C.bn_apply(z, a32, scale, shift, True)
    g = ops["gout"].clone()
    bpart = torch.zeros(C.bn_part_floats(N * 256, 64, True), device=dev)
    coef = torch.empty(4 * 64, device=dev)
    wpart = torch.empty(C.wgrad0_part_floats(N), device=dev)
    dg, db, dbias = (torch.zeros(64, device=dev) for _ in range(3))
    dw = torch.empty_like(ops["w"])
    sig = torch.zeros(1, dtype=torch.int32, device=dev)
    C.bn_bwd_wgrad0(g, 1, g, z, scale, shift, mean, invstd, ops["gamma"], bpart, coef, dg, db, dbias, ops["x"], wpart,
                    dw, sig=sig, sig_val=5)
    torch.cuda.synchronize()
    assert int(sig.item()) == 5
    assert _rel(mean, ref["mean"]) < 1e-5 and _rel(invstd, ref["invstd"]) < 1e-5
    assert _rel(rm, ref["rm"]) < 1e-5 and _rel(rv, ref["rv"]) < 1e-5 and int(nbt.item()) == 1
    assert _rel(a32, ref["a"]) < 1e-5
    assert _rel(planes.float().sum(0), ref["a"]) < 1e-5
    assert _rel(dg, ref["dgamma"]) < 2e-5, _rel(dg, ref["dgamma"])
    assert _rel(db, ref["dbeta"]) < 2e-5
    assert dbias.abs().max().item() < 1e-3 * ref["dbeta"].abs().max().item() + 1e-4  # analytically 0
    assert _rel(dw[..., :3].permute(0, 3, 1, 2), ref["dw"]) < 2e-5, _rel(dw[..., :3].permute(0, 3, 1, 2), ref["dw"])
    assert dw[..., 3:].abs().max().item() == 0.0 if CP > 3 else True
