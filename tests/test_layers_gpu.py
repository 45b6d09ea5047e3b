"""Generic NHWC autograd layers (ops/functional.py) on the GPU kernels vs fp64 torch references,
and a ResNet-50-shaped block / small ResNet training step through the native path."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def rel_norm(a, b):
    """||a-b|| / ||b||: robust to the few ReLU-mask flips that bf16-rounded inputs cause (a flipped
    element costs a full-size error in the max norm)."""
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("impl,tol", [("x3", 2e-5), ("bf16", 2e-2)])
@pytest.mark.parametrize("shape", [(4, 14, 14, 64, 64, 3, 2, 1), (4, 14, 14, 64, 256, 1, 1, 0),
                                   (4, 14, 14, 256, 128, 1, 2, 0), (2, 32, 32, 8, 64, 7, 2, 3)])
def test_conv2d_nhwc_fwd_bwd(shape, impl, tol):
    from distributed_pytorch_amd.ops.functional import conv2d_nhwc

    N, H, W, C, K, R, st, pd = shape
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, C, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(K, C, R, R, generator=g, dtype=torch.float64) * 0.1
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=st, padding=pd)
    dy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(dy)
    xd = x.permute(0, 2, 3, 1).float().contiguous().cuda().requires_grad_(True)
    wd = w.permute(0, 2, 3, 1).float().contiguous().cuda().requires_grad_(True)
    y = conv2d_nhwc(xd, wd, st, pd, impl)
    y.backward(dy.permute(0, 2, 3, 1).float().contiguous().cuda())
    torch.cuda.synchronize()
    assert rel(y.permute(0, 3, 1, 2), yr) < tol
    assert rel(xd.grad.permute(0, 3, 1, 2), xr.grad) < tol
    assert rel(wd.grad.permute(0, 3, 1, 2), wr.grad) < tol


@pytest.mark.parametrize("act", ["relu", "none", "add_relu"])
def test_bn_act_nhwc_fwd_bwd(act):
    from distributed_pytorch_amd.ops.functional import bn_act_nhwc

    g = torch.Generator().manual_seed(2)
    N, H, W, C = 8, 7, 7, 64
    z = torch.randn(N, H, W, C, generator=g, dtype=torch.float64) * 2 + 0.5
    gamma = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(C, generator=g, dtype=torch.float64)
    res = torch.randn(N, H, W, C, generator=g, dtype=torch.float64)
    zr, gr, br, rr = (t.clone().requires_grad_(True) for t in (z, gamma, beta, res))
    rm, rv = torch.zeros(C, dtype=torch.float64), torch.ones(C, dtype=torch.float64)
    u = F.batch_norm(zr.permute(0, 3, 1, 2), rm, rv, gr, br, True, 0.1, 1e-5).permute(0, 2, 3, 1)
    yr = {"relu": torch.relu(u), "none": u, "add_relu": torch.relu(u + rr)}[act]
    dy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(dy)
    c = lambda t: t.float().contiguous().cuda()
    zd, gd, bd, resd = (c(t).requires_grad_(True) for t in (z, gamma, beta, res))
    rmd, rvd = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    nbt = torch.zeros(1, dtype=torch.long, device="cuda")
    y = bn_act_nhwc(zd, gd, bd, rmd, rvd, nbt, True, 0.1, 1e-5, act, resd if act == "add_relu" else None)
    y.backward(c(dy))
    torch.cuda.synchronize()
    assert rel(y, yr) < 1e-5
    assert rel(zd.grad, zr.grad) < 1e-4
    assert rel(gd.grad, gr.grad) < 1e-4 and rel(bd.grad, br.grad) < 1e-4
    if act == "add_relu":
        assert rel(resd.grad, rr.grad) < 1e-5
    assert rel(rmd, rm) < 1e-5 and rel(rvd, rv) < 1e-5 and int(nbt.item()) == 1


def test_small_resnet_step_matches_reference():
    """A small ResNet built from the kernel layers (x3: fp32-grade) vs the stock-torch oracle."""
    from distributed_pytorch_amd.models.resnet import ResNet, ResNetRef

    torch.manual_seed(0)
    ours = ResNet([1, 1, 1, 1], 10, impl="x3").cuda()
    ref = ResNetRef([1, 1, 1, 1], 10).double()
    ref.load_state_dict({k: v.cpu() for k, v in ours.state_dict().items()})
    g = torch.Generator().manual_seed(3)
    x = torch.randn(8, 3, 64, 64, generator=g, dtype=torch.float64)
    t = torch.randint(0, 10, (8,), generator=g)
    lo = ours(x.permute(0, 2, 3, 1).float().contiguous().cuda())
    lr = ref(x)
    F.cross_entropy(lo, t.cuda()).backward()
    F.cross_entropy(lr, t).backward()
    torch.cuda.synchronize()
    assert rel(lo, lr) < 1e-3
    po = dict(ours.named_parameters())
    for name, p in ref.named_parameters():
        q = po[name].grad
        if q.dim() == 4:
            q = q[..., :p.shape[1]].permute(0, 3, 1, 2)
        assert rel(q, p.grad) < 2e-2, name


def test_resnet50_bf16_ddp_single_rank_trains():
    """ResNet-50 (bf16 kernels) through the generic DDP wrapper + fused SGD: loss decreases on a
    fixed batch (small image size to keep the test short)."""
    from distributed_pytorch_amd.models.resnet import resnet50
    from distributed_pytorch_amd.parallel.ddp import DistributedDataParallel, FlatSGD

    torch.manual_seed(0)
    m = resnet50(10, "bf16").cuda()
    ddp = DistributedDataParallel(m)
    opt = FlatSGD(ddp, lr=0.002, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(32, 64, 64, 3, device="cuda")
    t = torch.randint(0, 10, (32,), device="cuda")
    losses = []
    for _ in range(20):
        opt.zero_grad()
        loss = F.cross_entropy(ddp(x), t)
        loss.backward()
        opt.step(ddp.finish())
        losses.append(float(loss.item()))
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < 0.8 * losses[0], losses


def test_bf16_activation_path_dtypes_and_accuracy():
    """impl bf16: conv outputs / BN outputs / activation gradients are bf16 tensors produced directly
    by the kernels.  Each stage is checked against an fp64 reference fed with the SAME (bf16)
    inputs that stage received (end-to-end comparisons are dominated by ReLU-mask flips)."""
    from distributed_pytorch_amd.ops.functional import bn_act_nhwc, conv2d_nhwc

    g = torch.Generator().manual_seed(4)
    N, H, C, K = 8, 14, 64, 128
    x = torch.randn(N, H, H, C, generator=g).to(torch.bfloat16)
    w = torch.randn(K, 3, 3, C, generator=g) * 0.05
    dy = torch.randn(N, H, H, K, generator=g).to(torch.bfloat16)
    xd = x.cuda().requires_grad_(True)
    wd = w.cuda().requires_grad_(True)
    z = conv2d_nhwc(xd, wd, 1, 1, "bf16")
    z.retain_grad()
    assert z.dtype == torch.bfloat16
    rmd, rvd = torch.zeros(K, device="cuda"), torch.ones(K, device="cuda")
    a = bn_act_nhwc(z, torch.ones(K, device="cuda"), torch.zeros(K, device="cuda"), rmd, rvd, None, True, 0.1, 1e-5,
                    "relu")
    assert a.dtype == torch.bfloat16
    a.backward(dy.cuda())
    torch.cuda.synchronize()
    assert xd.grad.dtype == torch.bfloat16 and wd.grad.dtype == torch.float32
    nchw = lambda t: t.double().cpu().permute(0, 3, 1, 2)
    wb = nchw(w.to(torch.bfloat16))  # the kernel consumes the weight rounded to bf16
    # conv forward
    assert rel(nchw(z), F.conv2d(nchw(x), wb, padding=1)) < 1e-2
    # BN + ReLU forward/backward from our z
    zr = nchw(z.detach()).requires_grad_(True)
    ones, zeros = torch.ones(K, dtype=torch.float64), torch.zeros(K, dtype=torch.float64)
    yr = torch.relu(F.batch_norm(zr, None, None, ones, zeros, True, 0.1, 1e-5))
    yr.backward(nchw(dy))
    assert rel(nchw(a), yr) < 1e-2
    assert rel(nchw(z.grad), zr.grad) < 2e-2
    # conv backward from our dz
    dzr = nchw(z.grad)
    assert rel(nchw(xd.grad), torch.nn.grad.conv2d_input(list(nchw(x).shape), wb, dzr, padding=1)) < 1e-2
    assert rel(nchw(wd.grad), torch.nn.grad.conv2d_weight(nchw(x), list(wb.shape), dzr, padding=1)) < 1e-2
    assert rel(rmd, torch.zeros(K).double() * 0.9 + 0.1 * zr.detach().mean((0, 2, 3))) < 2e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,k,s,p", [((2, 112, 112, 64), 3, 2, 1), ((3, 9, 7, 16), 3, 2, 1),
                                         ((2, 8, 8, 8), 2, 2, 0), ((1, 10, 10, 24), 3, 1, 1)])
def test_maxpool_nhwc_matches_torch(shape, k, s, p, dtype):
    """Native NHWC max-pool (pool.hip) == torch max_pool2d forward and backward, including ties
    (first max in window scan order) and windows cut by the padding."""
    from distributed_pytorch_amd.ops import functional as Fn

    g = torch.Generator().manual_seed(31)
    x = torch.randn(shape, generator=g).round(decimals=1).to(dtype)  # rounding makes ties common
    xg = x.cuda().requires_grad_(True)
    y = Fn.max_pool_nhwc(xg, k, s, p)
    dy = torch.randn(y.shape, generator=g).to(dtype)
    (dx,) = torch.autograd.grad(y, xg, dy.cuda())
    xr = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p)
    (dxr,) = torch.autograd.grad(yr, xr, dy.double().permute(0, 3, 1, 2))
    assert torch.equal(y.cpu().double(), yr.detach().permute(0, 2, 3, 1))
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    assert (dx.cpu().double() - dxr.permute(0, 2, 3, 1)).abs().max() <= tol * dxr.abs().max()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 112, 112, 64), (3, 9, 7, 16), (1, 10, 10, 8), (2, 1, 2, 8)])
def test_maxpool_k3s2_backward_bitwise(monkeypatch, shape, dtype):
    """The 3x3/s2/p1 backward specialisation (2x2 input pixels per thread, each window loaded once)
    == the general gather, bitwise (same per-pixel summation order), ties included."""
    from distributed_pytorch_amd.ops import functional as Fn

    g = torch.Generator().manual_seed(12)
    x = torch.randn(shape, generator=g).round(decimals=1).to(dtype).cuda().requires_grad_(True)
    y = Fn.max_pool_nhwc(x, 3, 2, 1)
    dy = torch.randn(y.shape, generator=g).to(dtype).cuda()
    out = []
    for on in ("0", "1"):
        monkeypatch.setenv("DPA_POOL_K3S2", on)
        (dx,) = torch.autograd.grad(y, x, dy, retain_graph=True)
        torch.cuda.synchronize()
        out.append(dx.view(torch.int16) if dtype == torch.bfloat16 else dx)
    assert torch.equal(out[0], out[1])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape,pool", [((4, 16, 16, 64), (3, 2, 1)), ((2, 15, 17, 16), (3, 2, 1)),
                                        ((2, 8, 8, 8), (2, 2, 0))])
def test_bn_relu_maxpool_fused_bitwise(monkeypatch, shape, pool, dtype):
    """BN + ReLU applied in the max-pool's loads (bn_act_nhwc ``pool``, the ResNet stem) == the BN
    apply pass followed by the pool: output, running statistics and every gradient bitwise."""
    from distributed_pytorch_amd.ops import functional as Fn

    g = torch.Generator().manual_seed(5)
    C = shape[-1]
    z0 = (torch.randn(shape, generator=g) * 2 + 0.3).round(decimals=1).to(dtype).cuda()  # ties are common
    gm0, bt0 = (torch.rand(C, generator=g) + 0.5).cuda(), (torch.randn(C, generator=g) * 0.2).cuda()
    dy = None

    def run(fused):
        nonlocal dy
        monkeypatch.setattr(Fn, "FUSE_BN_POOL", fused)
        z = z0.clone().requires_grad_(True)
        gm, bt = gm0.clone().requires_grad_(True), bt0.clone().requires_grad_(True)
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        nbt = torch.zeros(1, dtype=torch.long, device="cuda")
        y = Fn.bn_act_nhwc(z, gm, bt, rm, rv, nbt, True, 0.1, 1e-5, "relu", pool=pool)
        if dy is None:
            dy = torch.randn(y.shape, generator=g).to(dtype).cuda()
        y.backward(dy)
        torch.cuda.synchronize()
        return y, z.grad, gm.grad, bt.grad, rm, rv

    ref, fused = run(False), run(True)
    for a, b in zip(ref, fused):
        assert a.shape == b.shape and torch.equal(a.view(-1).view(torch.int16) if a.dtype == torch.bfloat16 else a,
                                                  b.view(-1).view(torch.int16) if b.dtype == torch.bfloat16 else b)


@pytest.mark.parametrize("cin,width,stride,hw", [(64, 64, 1, 14), (256, 128, 2, 14), (64, 32, 2, 9)])
def test_downsample_bn_fused_into_add_bitwise(monkeypatch, cin, width, stride, hw):
    """A bottleneck with a downsample branch: its BN applied inside bn3's add + ReLU (bn_act_nhwc
    ``res_bn``, no stored BN output) == the separate BN pass: output, input gradient, every parameter
    gradient and the running statistics bitwise."""
    from distributed_pytorch_amd.models.resnet import Bottleneck
    from distributed_pytorch_amd.ops import functional as Fn

    torch.manual_seed(3)
    ref = Bottleneck(cin, width, stride, True, "bf16").cuda()
    g = torch.Generator().manual_seed(4)
    x0 = torch.randn(4, hw, hw, cin, generator=g).to(torch.bfloat16).cuda()
    dy = None

    def run(fused):
        nonlocal dy
        monkeypatch.setattr(Fn, "FUSE_RES_BN", fused)
        m = Bottleneck(cin, width, stride, True, "bf16").cuda()
        m.load_state_dict(ref.state_dict())
        x = x0.clone().requires_grad_(True)
        y = m(x)
        if dy is None:
            dy = torch.randn(y.shape, generator=g).to(torch.bfloat16).cuda()
        y.backward(dy)
        torch.cuda.synchronize()
        grads = [p.grad for _, p in sorted(m.named_parameters())]
        bufs = [b for _, b in sorted(m.named_buffers())]
        return [y, x.grad] + grads + bufs

    a, b = run(False), run(True)
    assert len(a) == len(b)
    for u, v in zip(a, b):
        assert u is not None and v is not None and u.shape == v.shape
        assert torch.equal(u.view(-1).view(torch.int16) if u.dtype == torch.bfloat16 else u,
                           v.view(-1).view(torch.int16) if v.dtype == torch.bfloat16 else v)


def test_head_kernels_match_torch():
    """GAP + Linear + softmax-CE head (head.hip + hipBLASLt GEMMs) vs torch fp64: loss, dx (bf16),
    dW, db; and the logits head's backward."""
    from distributed_pytorch_amd.ops import functional as Fn

    g = torch.Generator().manual_seed(8)
    N, H, C, J = 16, 7, 256, 100
    x = torch.randn(N, H, H, C, generator=g).to(torch.bfloat16)
    w = torch.randn(J, C, generator=g) * 0.05
    b = torch.randn(J, generator=g) * 0.1
    t = torch.randint(0, J, (N,), generator=g)
    xr, wr, br = x.double().requires_grad_(True), w.double().requires_grad_(True), b.double().requires_grad_(True)
    lr = F.cross_entropy(xr.mean(dim=(1, 2)) @ wr.t() + br, t)
    (3.0 * lr).backward()
    xd, wd, bd = x.cuda().requires_grad_(True), w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    lo = Fn.head_ce(xd, wd, bd, t.cuda())
    (3.0 * lo).backward()
    torch.cuda.synchronize()
    assert abs(lo.item() - lr.item()) < 1e-5 * max(1, abs(lr.item()))
    assert xd.grad.dtype == torch.bfloat16
    assert rel(xd.grad, xr.grad) < 1e-2 and rel(wd.grad, wr.grad) < 1e-5 and rel(bd.grad, br.grad) < 1e-5
    # logits form, own loss
    xd.grad = wd.grad = bd.grad = None
    lg = Fn.head_logits(xd, wd, bd)
    F.cross_entropy(lg, t.cuda()).mul(3.0).backward()
    torch.cuda.synchronize()
    assert rel(wd.grad, wr.grad) < 1e-5 and rel(bd.grad, br.grad) < 1e-5 and rel(xd.grad, xr.grad) < 1e-2


def test_resnet_fused_loss_step_matches_reference():
    """Small ResNet (x3) trained through model(x, target) -- fused head, GradJoin residual sums,
    channel padding in the plane split -- against (a) the same network through the logits head +
    stock cross_entropy + autograd's own residual sums, which must agree to fp32 rounding, and (b) the
    stock-torch oracle in fp64.  Against fp64 a few tensors of a random-init network sit behind a
    ReLU whose input is ~0 at some element: fp32 rounding flips that mask bit (stock torch fp32 does
    too), so (b) bounds the median tensor tightly and every tensor loosely."""
    from distributed_pytorch_amd.models import resnet as R

    torch.manual_seed(0)
    base = R.ResNet([1, 2, 1, 1], 10, impl="x3")
    sd = base.state_dict()
    ref = R.ResNetRef([1, 2, 1, 1], 10).double()
    ref.load_state_dict(sd)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(8, 3, 64, 64, generator=g, dtype=torch.float64)
    t = torch.randint(0, 10, (8,), generator=g)
    lr = F.cross_entropy(ref(x), t)
    lr.backward()
    xin = x.permute(0, 2, 3, 1).float().contiguous().cuda()
    grads = []
    for fused in (True, False):
        m = R.ResNet([1, 2, 1, 1], 10, impl="x3")
        m.load_state_dict(sd)
        m = m.cuda()
        if not fused:  # logits head + stock loss, residual gradients summed by autograd
            class PassThrough(R.Fn.GradJoin):
                __slots__ = ()

                def last(self):
                    return False

                def contribute(self, gr):  # every contribution goes to autograd
                    return gr

            for blk in m.modules():
                if isinstance(blk, R.Bottleneck):
                    blk._join = PassThrough(2)
        lo = m(xin, t.cuda()) if fused else F.cross_entropy(m(xin), t.cuda())
        lo.backward()
        torch.cuda.synchronize()
        assert abs(lo.item() - lr.item()) < 1e-4 * max(1.0, abs(lr.item()))
        grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
    errs = []
    for name, p in ref.named_parameters():
        a, b = grads[0][name], grads[1][name]
        assert rel(a, b) < 1e-5, name
        q = a[..., :p.shape[1]].permute(0, 3, 1, 2) if a.dim() == 4 else a
        e = rel(q, p.grad)
        assert e < 0.2, name
        errs.append(e)
    errs.sort()
    assert errs[len(errs) // 2] < 5e-3, errs


@pytest.mark.parametrize("impl", ["x3", "bf16"])
def test_resnet_deferred_residual_gradient(monkeypatch, impl):
    """A block input's second gradient contribution left to the producing BN backward (summed on
    load, bn.hip g2) instead of an add pass.  x3: gradients bitwise those of the add-pass path (both
    add in fp32).  bf16: the add pass rounds the sum to bf16 and the deferred path does not, so the
    two differ by bf16 rounding propagated through the network; both are compared with the x3
    (fp32-grade) gradients, and the deferred path must be no less accurate."""
    from distributed_pytorch_amd.models import resnet as R

    torch.manual_seed(0)
    sd = R.ResNet([1, 3, 1, 1], 10, impl=impl).state_dict()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(8, 64, 64, 3, generator=g).cuda()
    t = torch.randint(0, 10, (8,), generator=g).cuda()

    def run(impl_, defer):
        monkeypatch.setattr(R.Fn, "DEFER_JOIN", defer)
        m = R.ResNet([1, 3, 1, 1], 10, impl=impl_)
        m.load_state_dict(sd)
        m = m.cuda()
        n0 = R.Fn.DEFER_STATS["summed_on_load"]
        m(x, t).backward()
        torch.cuda.synchronize()
        used = R.Fn.DEFER_STATS["summed_on_load"] - n0
        assert (used > 0) == defer, used
        assert not R.Fn._DEFERRED
        return {n: p.grad.detach().float().clone() for n, p in m.named_parameters()}

    add_pass, deferred = run(impl, False), run(impl, True)
    if impl == "x3":
        for n in add_pass:
            assert torch.equal(add_pass[n], deferred[n]), n
        return
    ref = run("x3", False)
    e_add = sorted(rel(add_pass[n], ref[n]) for n in ref)
    e_def = sorted(rel(deferred[n], ref[n]) for n in ref)
    med = len(ref) // 2
    assert e_def[med] <= 1.25 * e_add[med] + 1e-3, (e_def[med], e_add[med])
    assert e_def[-1] <= 1.5 * e_add[-1] + 1e-2, (e_def[-1], e_add[-1])


@pytest.mark.parametrize("impl", ["x3", "bf16"])
def test_resnet_relu_mask_matches_residual_recompute(monkeypatch, impl):
    """The add+ReLU BN backward reading the forward's ReLU mask (1 byte per 4 channels) instead of
    re-reading the residual: the mask is the comparison the backward would recompute, so the
    gradients are bitwise identical."""
    from distributed_pytorch_amd.models import resnet as R

    torch.manual_seed(0)
    sd = R.ResNet([1, 2, 1, 1], 10, impl=impl).state_dict()
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8, 64, 64, 3, generator=g).cuda()
    t = torch.randint(0, 10, (8,), generator=g).cuda()
    grads = []
    for use_mask in (False, True):
        monkeypatch.setattr(R.Fn, "BN_RELU_MASK", use_mask)
        m = R.ResNet([1, 2, 1, 1], 10, impl=impl)
        m.load_state_dict(sd)
        m = m.cuda()
        m(x, t).backward()
        torch.cuda.synchronize()
        grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
    for n in grads[0]:
        assert torch.equal(grads[0][n], grads[1][n]), n


@pytest.mark.parametrize("impl", ["x3", "bf16"])
def test_resnet_epilogue_bn_stats(monkeypatch, impl):
    """BN statistics from the producing conv's epilogue (functional.EPI_STATS) vs the statistics pass:
    the forward BNs really take the epilogue path, the running statistics agree to fp32 rounding
    and the loss and gradients within the conditioning of a batch-8 step."""
    from distributed_pytorch_amd.models import resnet as R

    torch.manual_seed(0)
    sd = R.ResNet([1, 2, 1, 1], 10, impl=impl).state_dict()
    g = torch.Generator().manual_seed(8)
    x = torch.randn(8, 64, 64, 3, generator=g).cuda()
    t = torch.randint(0, 10, (8,), generator=g).cuda()
    out = []
    for epi in (False, True):
        monkeypatch.setattr(R.Fn, "EPI_STATS", epi)
        m = R.ResNet([1, 2, 1, 1], 10, impl=impl)
        m.load_state_dict(sd)
        m = m.cuda()
        used0 = R.Fn.STATS_USED["epilogue"]
        loss = m(x, t)
        loss.backward()
        torch.cuda.synchronize()
        used = R.Fn.STATS_USED["epilogue"] - used0
        assert (used > 0) == epi, used
        out.append((loss.item(), {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()},
                    {n: b.detach().double().cpu() for n, b in m.named_buffers() if "running" in n}))
    # batch 8: the BN statistics of a few samples make the gradients ill-conditioned (ReLU / max-pool
    # decisions flip on last-bit changes), the bounds of test_small_resnet_step_matches_reference
    # (bf16: rounding flips make the gradients chaotic at this size; the loss and statistics are
    # compared, the gradient numerics are checked through x3)
    tol = 2e-2
    assert abs(out[0][0] - out[1][0]) <= (1e-3 if impl == "x3" else 1e-2) * abs(out[0][0])
    for n in (out[0][1] if impl == "x3" else ()):
        a, b = out[0][1][n], out[1][1][n]
        assert (a - b).abs().max().item() <= tol * max(a.abs().max().item(), 1e-6), n
    for n in (out[0][2] if impl == "x3" else ()):  # bf16: a last-bit statistics change moves the next
        a, b = out[0][2][n], out[1][2][n]             # layer's bf16 input roundings
        assert (a - b).abs().max().item() <= 1e-4 * max(a.abs().max().item(), 1e-6), n


def test_eval_no_grad_registers_no_epilogue_stats():
    """An eval forward under no_grad (parameters still requiring grad) registers no epilogue BN
    statistics: eval-mode BN never pops them, and each entry pins its conv output."""
    from distributed_pytorch_amd.models import resnet as R

    torch.manual_seed(0)
    m = R.ResNet([1, 1, 1, 1], 10, impl="x3").cuda()
    x = torch.randn(4, 64, 64, 3).cuda()
    t = torch.randint(0, 10, (4,)).cuda()
    m(x, t).backward()  # a training step first (clears and repopulates the table)
    torch.cuda.synchronize()
    R.Fn._STATS.clear()
    m.eval()
    with torch.no_grad():
        m(x, t)
    torch.cuda.synchronize()
    assert len(R.Fn._STATS) == 0


def test_resnet_graph_replay_matches_eager():
    """bench_resnet.py --graph: a whole ResNet training step (forward, autograd backward through the
    native kernels, DDP hooks, fused SGD) captured once and replayed gives bitwise the parameters of
    the same number of eager steps."""
    from distributed_pytorch_amd.models import resnet as R
    from distributed_pytorch_amd.parallel.ddp import DistributedDataParallel, FlatSGD

    torch.manual_seed(0)
    sd = R.ResNet([1, 2, 1, 1], 10, impl="bf16").state_dict()
    g = torch.Generator().manual_seed(10)
    x = torch.randn(16, 64, 64, 3, generator=g).cuda()
    t = torch.randint(0, 10, (16,), generator=g).cuda()
    out = []
    for graph in (False, True):
        m = R.ResNet([1, 2, 1, 1], 10, impl="bf16")
        m.load_state_dict(sd)
        ddp = DistributedDataParallel(m.cuda())
        opt = FlatSGD(ddp, lr=0.05, momentum=0.9, weight_decay=1e-4)
        one = torch.ones((), device="cuda")

        def step():
            opt.zero_grad()
            loss = ddp(x, t)
            loss.backward(one)
            opt.step(ddp.finish())
            return loss

        if not graph:
            for _ in range(5):
                step()
        else:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(2):
                    step()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                step()
            for _ in range(3):
                gr.replay()
        torch.cuda.synchronize()
        out.append(ddp.flat_params.detach().clone())
    assert torch.isfinite(out[0]).all()
    assert torch.equal(out[0], out[1])


