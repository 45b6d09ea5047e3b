"""HIP kernels (BN activation variants, classifier head, SGD, augmentation) vs the plain-PyTorch
fp32 reference of the same op (distributed_pytorch_amd.ops.cpu_ref mirrors the native API), and one
whole VGG-11 training step of the GPU engine vs stock torch autograd on model.VGG11.  The VGG
BatchNorm+ReLU+max-pool kernels are checked against torch autograd in fp64 in test_bn_gpu.py."""
import pytest
import torch
import torch.nn.functional as F

from distributed_pytorch_amd.ops import cpu_ref

pytestmark = pytest.mark.gpu


def _C():
    from distributed_pytorch_amd import _ext

    return _ext.require()


def close(a, b, tol):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    d = (a - b).abs().max().item()
    s = b.abs().max().clamp_min(1e-6).item()
    assert d <= tol * s, f"max abs diff {d} vs scale {s}"


@pytest.mark.parametrize("act", [0, 1, 2])
def test_bn_backward_wide_geometry(act):
    """BN backward of a tensor large enough for the 1024-thread reduce geometry (> 3M float4 lanes,
    ResNet-50-sized: two rows' loads in flight), activation/residual variants, vs the fp32 reference."""
    C_ = _C()
    N, H, W, C = 16, 56, 56, 256
    g = torch.Generator().manual_seed(11 + act)
    z = torch.randn(N, H, W, C, generator=g)
    gamma, beta = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.5
    mean, invstd = z.reshape(-1, C).mean(0), torch.rsqrt(z.reshape(-1, C).var(0, unbiased=False) + 1e-5)
    scale, shift = gamma * invstd, beta - mean * gamma * invstd
    gout = torch.randn(N, H, W, C, generator=g)
    res = torch.randn(N, H, W, C, generator=g) if act == 2 else None
    ref = [torch.zeros(C) for _ in range(3)]
    dz_ref = torch.empty_like(z)
    dres_ref = torch.empty_like(z) if act == 2 else None
    cpu_ref.bn_bwd(gout, 1, gout, z, scale, shift, mean, invstd, gamma, None, None, ref[0], ref[1], ref[2], dz_ref,
                   False, act, res, dres_ref)
    d = lambda t: t.cuda()
    part = torch.zeros(C_.bn_part_floats(N * H * W, C, True), device="cuda")
    coef = torch.empty(4 * C, device="cuda")
    out = [torch.zeros(C, device="cuda") for _ in range(3)]
    dz = torch.empty(z.shape, device="cuda")
    dres = torch.empty(z.shape, device="cuda") if act == 2 else None
    gd = d(gout)
    C_.bn_bwd(gd, 1, gd, d(z), d(scale), d(shift), d(mean), d(invstd), d(gamma), part, coef, out[0], out[1], out[2],
              dz, False, act, d(res) if res is not None else None, dres)
    torch.cuda.synchronize()
    close(dz, dz_ref, 2e-5)
    close(out[0], ref[0], 2e-5)
    close(out[1], ref[1], 2e-5)
    if act == 2:
        close(dres, dres_ref, 1e-6)


def test_bn_backward_matches_torch_autograd():
    """End-to-end oracle: torch's own BatchNorm2d(train)+ReLU+MaxPool backward (fp64)."""
    C_ = _C()
    N, H, W, C = 8, 8, 8, 64
    g = torch.Generator().manual_seed(2)
    x = torch.randn(N, C, H, W, generator=g, dtype=torch.float64).requires_grad_(True)
    bn = torch.nn.BatchNorm2d(C).double()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_()
    y = F.max_pool2d(torch.relu(bn(x)), 2, 2)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    gx, gw, gb = torch.autograd.grad(y, (x, bn.weight, bn.bias), gy)
    z = x.detach().float().permute(0, 2, 3, 1).contiguous()
    mean = z.reshape(-1, C).mean(0)
    invstd = torch.rsqrt(z.reshape(-1, C).var(0, unbiased=False) + 1e-5)
    gamma, beta = bn.weight.detach().float(), bn.bias.detach().float()
    scale = gamma * invstd
    shift = beta - mean * scale
    d = lambda t: t.contiguous().cuda()
    out = [torch.zeros(C, device="cuda") for _ in range(3)]
    dz = torch.empty(z.shape, device="cuda")
    part = torch.zeros(C_.bn_part_floats(N * H * W // 4, C, True), device="cuda")
    coef = torch.empty(4 * C, device="cuda")
    gg = d(gy.float().permute(0, 2, 3, 1))
    C_.bn_bwd(gg, 1, gg, d(z), d(scale), d(shift), d(mean), d(invstd), d(gamma), part, coef,
              out[0], out[1], out[2], dz, True)
    torch.cuda.synchronize()
    close(dz.permute(0, 3, 1, 2), gx, 1e-4)
    close(out[0], gw, 1e-4)
    close(out[1], gb, 1e-4)


@pytest.mark.parametrize("B,Cin,J", [(256, 512, 10), (7, 64, 3), (33, 100, 16)])
def test_fc_ce(B, Cin, J):
    C_ = _C()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, Cin, generator=g)
    w = torch.randn(J, Cin, generator=g) * 0.1
    b = torch.randn(J, generator=g)
    t = torch.randint(0, J, (B,), generator=g)
    xr, wr, br = x.double().requires_grad_(True), w.double().requires_grad_(True), b.double().requires_grad_(True)
    loss = F.cross_entropy(xr @ wr.t() + br, t)
    gx, gw, gb = torch.autograd.grad(loss, (xr, wr, br))
    d = lambda z: z.cuda()
    lr_, dl, dx = torch.empty(B, device="cuda"), torch.empty(B, J, device="cuda"), torch.empty(B, Cin, device="cuda")
    dw, db, lo, acc = torch.empty(J, Cin, device="cuda"), torch.empty(J, device="cuda"), torch.zeros(1, device="cuda"), \
        torch.zeros(1, device="cuda")
    C_.fc_ce_train(d(x), d(w), d(b), d(t), lr_, dl, dx, dw, db, lo, acc)
    torch.cuda.synchronize()
    close(lo, loss.detach(), 1e-5)
    close(acc, loss.detach(), 1e-5)
    close(dx, gx, 1e-5)
    close(dw, gw, 1e-5)
    close(db, gb, 1e-5)
    corr = torch.empty(B, dtype=torch.int32, device="cuda")
    ev = torch.zeros(2, device="cuda")
    C_.fc_ce_eval(d(x), d(w), d(b), d(t), lr_, corr, None, ev)
    torch.cuda.synchronize()
    pred = (x.double() @ w.double().t() + b.double()).argmax(1)
    assert int(ev[1].item()) == int((pred == t).sum())
    close(ev[0:1], loss.detach().reshape(1), 1e-5)


@pytest.mark.parametrize("np_", [1, 3])
def test_sgd_flat_writes_planes(np_):
    """The fused update also refreshes the bf16 operand planes of the updated slice (only)."""
    C_ = _C()
    n = 8192
    g = torch.Generator().manual_seed(5)
    p, gr, m = torch.randn(n, generator=g), torch.randn(n, generator=g), torch.randn(n, generator=g)
    pr, mr = p.clone(), m.clone()
    cpu_ref.sgd_flat(pr, gr, mr, 0.1, 0.9, 1e-4, 1.0, False, 1024, 4096)
    pd, md = p.cuda(), m.cuda()
    planes = torch.zeros(np_, n, device="cuda", dtype=torch.bfloat16)
    C_.sgd_flat(pd, gr.cuda(), md, 0.1, 0.9, 1e-4, 1.0, False, 1024, 4096, planes)
    torch.cuda.synchronize()
    close(pd, pr, 1e-6)
    # planes are the exact RNE split of the kernel's own updated parameters
    assert torch.equal(planes.cpu()[:, 1024:5120], cpu_ref.split_bf16(pd.cpu()[1024:5120], np_))
    assert planes[:, :1024].abs().sum().item() == 0 and planes[:, 5120:].abs().sum().item() == 0
    # the planes reconstruct the updated fp32 parameters
    rec = planes.double().sum(0).cpu()[1024:5120]
    tol = 2 ** -22 if np_ == 3 else 2 ** -8
    assert ((rec - pd.double().cpu()[1024:5120]).abs() / pd.double().cpu()[1024:5120].abs()).max() < tol


@pytest.mark.parametrize("first", [True, False])
def test_sgd_flat(first):
    C_ = _C()
    n = 4096 + 64
    g = torch.Generator().manual_seed(4)
    p, gr, m = torch.randn(n, generator=g), torch.randn(n, generator=g), torch.randn(n, generator=g)
    pr, mr = p.clone(), m.clone()
    cpu_ref.sgd_flat(pr, gr, mr, 0.1, 0.9, 1e-4, 0.5, first)
    pd, md = p.cuda(), m.cuda()
    C_.sgd_flat(pd, gr.cuda(), md, 0.1, 0.9, 1e-4, 0.5, first)
    torch.cuda.synchronize()
    close(pd, pr, 1e-6)
    close(md, mr, 1e-6)
    # reference torch.optim.SGD semantics
    pt = torch.nn.Parameter(p.clone())
    opt = torch.optim.SGD([pt], lr=0.1, momentum=0.9, weight_decay=1e-4)
    if not first:
        opt.state[pt]["momentum_buffer"] = m.clone()
    pt.grad = gr * 0.5
    opt.step()
    close(pd, pt.detach(), 1e-6)


def test_augment_matches_reference():
    C_ = _C()
    g = torch.Generator().manual_seed(5)
    imgs = torch.randint(0, 256, (50, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (50,), generator=g)
    idx = torch.randint(0, 50, (17,), generator=g)
    from distributed_pytorch_amd.data import MEAN, STD

    for train in (True, False):
        ref = torch.empty(17, 32, 32, 4)
        tr = torch.empty(17, dtype=torch.int64)
        cpu_ref.augment(imgs, idx, labels, ref, tr, 4, train, 99, 12345, MEAN, STD)
        out = torch.empty(17, 32, 32, 4, device="cuda")
        td = torch.empty(17, dtype=torch.int64, device="cuda")
        C_.augment(imgs.cuda(), idx.cuda(), labels.cuda(), out, td, 4, train, 99, 12345, MEAN, STD)
        torch.cuda.synchronize()
        close(out, ref, 1e-6)
        assert torch.equal(td.cpu(), tr)


@pytest.mark.parametrize("impl", ["fp32", "x3", "h2"])
def test_engine_step_matches_torch(impl):
    """One full training step (fwd, CE, bwd) of the HIP engine vs torch autograd (fp64) on the
    reference module, from the same weights and data.  Both fp32 paths must match to fp32-level."""
    from distributed_pytorch_amd.engine import VGGEngine
    from distributed_pytorch_amd.models import VGG11

    torch.manual_seed(1)
    m = VGG11().double()
    N = 32
    x = torch.randn(N, 3, 32, 32, dtype=torch.float64)
    t = torch.randint(0, 10, (N,))
    e = VGGEngine("VGG11", "cuda", max_batch=N, impl=impl)
    e.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in m.state_dict().items()})
    loss = F.cross_entropy(m(x), t)
    loss.backward()
    x4 = torch.zeros(N, 32, 32, 4)
    x4[..., :3] = x.float().permute(0, 2, 3, 1)
    l2 = e.forward_backward(x4.cuda(), t.cuda())
    torch.cuda.synchronize()
    assert abs(l2.item() - loss.item()) < 1e-4 * max(1.0, abs(loss.item()))
    for n, p in m.named_parameters():
        gref = p.grad
        gd = e._to_torch_layout(n, e.grads[n]).cpu()
        tol = 2e-3 if n.endswith("bias") and p.dim() == 1 and "layers" in n and gref.abs().max() < 1e-6 else 1e-3
        if gref.abs().max() < 1e-6:  # conv bias grads are analytically 0 (BN follows)
            assert gd.abs().max().item() < 1e-4
            continue
        close(gd, gref, tol)
    sd = e.state_dict()
    for k, v in m.state_dict().items():
        if "running" in k:
            close(sd[k], v, 1e-4)


def test_engine_trajectory_tracks_fp64():
    """Eight SGD steps (lr 0.1, momentum 0.9, wd 1e-4) of the x3 engine vs torch fp64 autograd +
    torch.optim.SGD from the same weights on the same batches: the loss trajectory and the final
    parameters stay within a small factor of stock torch fp32's own distance from fp64."""
    from distributed_pytorch_amd.engine import VGGEngine
    from distributed_pytorch_amd.models import VGG11

    torch.manual_seed(3)
    ref = VGG11().double()
    sd0 = {k: v.clone() for k, v in ref.state_dict().items()}
    g = torch.Generator().manual_seed(9)
    N, S = 64, 8
    xs = [torch.randn(N, 3, 32, 32, generator=g, dtype=torch.float64) for _ in range(S)]
    ts = [torch.randint(0, 10, (N,), generator=g) for _ in range(S)]

    def torch_run(dtype, dev):
        m = VGG11().to(dev, dtype)
        m.load_state_dict({k: v.to(dtype) if v.is_floating_point() else v for k, v in sd0.items()})
        opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        losses = []
        for x, t in zip(xs, ts):
            opt.zero_grad()
            loss = F.cross_entropy(m(x.to(dev, dtype)), t.to(dev))
            loss.backward()
            opt.step()
            losses.append(float(loss))
        return losses, {n: p.detach().double().cpu() for n, p in m.named_parameters()}

    l64, p64 = torch_run(torch.float64, "cpu")
    l32, p32 = torch_run(torch.float32, "cpu")
    e = VGGEngine("VGG11", "cuda", max_batch=N, impl="x3", lr=0.1)
    e.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in sd0.items()})
    le = []
    for x, t in zip(xs, ts):
        x4 = torch.zeros(N, 32, 32, 4)
        x4[..., :3] = x.float().permute(0, 2, 3, 1)
        e.forward_backward(x4.cuda(), t.cuda())
        e.sgd_step()
        e.finish_step()
        le.append(float(e.loss.item()))
    pe = {n: e._to_torch_layout(n, e.params[n]).cpu().double() for n in p64}

    def dist(p):
        num = sum(float((p[n] - p64[n]).norm() ** 2) for n in p64) ** 0.5
        return num / sum(float(v.norm() ** 2) for v in p64.values()) ** 0.5

    d32, de = dist(p32), dist(pe)
    assert de <= 4.0 * d32 + 1e-6, (de, d32)
    for a, b, c in zip(le, l32, l64):
        assert abs(a - c) <= 4.0 * abs(b - c) + 1e-4 * abs(c), (le, l32, l64)


@pytest.mark.parametrize("impl", ["fp32", "x3", "bf16", "h2"])
def test_engine_training_converges_and_evaluates(impl):
    """A few steps on a learnable synthetic set: loss goes down, eval runs, x3 tracks fp32 closely."""
    from distributed_pytorch_amd.data import DeviceLoader, ShardSampler, synthetic_cifar
    from distributed_pytorch_amd.engine import VGGEngine

    ds = synthetic_cifar(2048, 0)
    ld = DeviceLoader(ds, 128, "cuda", sampler=ShardSampler(2048, 1, 0), train=True, seed=1)
    e = VGGEngine("VGG11", "cuda", max_batch=128, impl=impl, lr=0.05)
    e.init_parameters(seed=1)
    losses = []
    for ep in range(2):
        ld.set_epoch(ep)
        for x, t in ld:
            e.forward_backward(x, t)
            e.sgd_step()
            e.finish_step()
            losses.append(float(e.loss.item()))
    assert all(l == l for l in losses)
    assert sum(losses[-4:]) / 4 < sum(losses[:4]) / 4
    e.begin_eval()
    for x, t in DeviceLoader(synthetic_cifar(256, 1), 128, "cuda", train=False):
        e.eval_batch(x, t)
    acc = e.eval_acc.cpu()
    assert 0 <= acc[1] <= 256 and acc[0] == acc[0]


@pytest.mark.parametrize("debug_sync", [False, True])
@pytest.mark.parametrize("mode", ["ddp", "allreduce", "gather", "zero1"])
def test_sync_modes_through_native_rccl_single_rank(mode, debug_sync, monkeypatch):
    """A 1-rank native RCCL communicator (every collective is an identity) driving the real
    bucket / comm-stream / event path: results must equal the no-communication run bit for bit."""
    from distributed_pytorch_amd import _ext
    from distributed_pytorch_amd.engine import VGGEngine
    from distributed_pytorch_amd.parallel import NullComm, RcclComm, make_sync

    if debug_sync:  # every collective host-synchronous + error-checked
        monkeypatch.setenv("DPA_DEBUG_SYNC", "1")
    C = _ext.require()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(9)
    xs = [torch.randn(32, 32, 32, 4, generator=g) for _ in range(3)]
    ts = [torch.randint(0, 10, (32,), generator=g) for _ in range(3)]
    outs = []
    # null comm with the update after backward, null comm with the per-bucket update fused into
    # backward (wgrad stream), 1-rank RCCL with the fused update on the comm stream, and 1-rank RCCL
    # with the default single update after backward
    runs = [(NullComm(), "0"), (NullComm(), "1"), (RcclComm(0, 1, dev, uid=C.rccl_unique_id()), "1"),
            (lambda: RcclComm(0, 1, dev, uid=C.rccl_unique_id()), "0")]
    for comm, fused in runs:
        comm = comm() if callable(comm) else comm
        monkeypatch.setenv("DPA_FUSED_STEP", fused)
        e = VGGEngine("VGG11", dev, max_batch=32, impl="x3", lr=0.01)
        e.init_parameters(seed=3)
        sync = make_sync(mode, e, comm, bucket_mb=1.0 if mode == "ddp" else None)
        for x, t in zip(xs, ts):
            x = x.cuda()
            x[..., 3] = 0
            sync.begin_step()
            e.forward_backward(x, t.cuda(), grad_ready=sync.grad_ready, pre_forward=sync.pre_forward,
                               params_free=sync.params_free)
            sync.update(sync.finish())
            e.finish_step()
        torch.cuda.synchronize()
        comm.check()
        outs.append(e.params.flat.clone())
        comm.close()
    assert all(torch.equal(outs[0], o) for o in outs[1:])


def test_bn_reductions_bitwise_reproducible():
    """BN statistics / backward sums use fixed-order merges: repeated launches on a shared
    workspace (interleaving shapes) give bitwise-identical results."""
    C_ = _C()
    shapes = [(256, 32, 32, 64), (256, 2, 2, 512), (64, 8, 8, 256), (3, 5, 7, 12)]
    need = max(C_.bn_part_floats(n * h * w, c, bwd) for n, h, w, c in shapes for bwd in (False, True))
    part = torch.zeros(need, device="cuda")
    results = {}
    for rep in range(3):
        for n, h, w, c in shapes:
            z = (torch.randn(n, h, w, c, generator=torch.Generator().manual_seed(n * c)) * 2 + 1).cuda()
            gamma, beta = torch.ones(c, device="cuda"), torch.zeros(c, device="cuda")
            outs = [torch.zeros(c, device="cuda") for _ in range(4)]
            C_.bn_fwd_stats(z, 1, z, part, gamma, beta, None, None, None, None, *outs, 0.1, 1e-5)
            zz = z.reshape(-1, c).double()
            close(outs[0], zz.mean(0).float(), 1e-5)
            close(outs[1], torch.rsqrt(zz.var(0, unbiased=False) + 1e-5).float(), 1e-4)
            cur = torch.cat(outs).cpu()
            key = (n, h, w, c)
            if key in results:
                assert torch.equal(cur, results[key])
            results[key] = cur


def test_rccl_watchdog_tracks_and_retires_ops():
    import time

    from distributed_pytorch_amd import _ext

    C = _ext.require()
    c = C.RcclComm(0, 1, C.rccl_unique_id(), 0, timeout_s=60.0, poll_s=0.05, exit_on_error=False)
    t = torch.ones(1 << 20, device="cuda")
    for _ in range(5):
        c.all_reduce(t, "sum")
    c.broadcast(t, 0)
    c.synchronize()
    deadline = time.time() + 10
    while c.outstanding() and time.time() < deadline:
        time.sleep(0.05)
    assert c.outstanding() == 0 and c.ops_issued() == 6
    assert c.async_error() == ""
    assert torch.all(t == 1)
    c.abort()
    with pytest.raises(RuntimeError, match="aborted"):
        c.all_reduce(t, "sum")


@pytest.mark.parametrize("impl", ["fp32", "x3", "h2"])
def test_engine_eval_matches_torch_after_training(impl):
    """After real training steps (running stats moved, weights updated), the engine's eval forward
    equals stock torch eval on its exported state_dict."""
    from distributed_pytorch_amd.data import DeviceLoader, ShardSampler, synthetic_cifar
    from distributed_pytorch_amd.engine import VGGEngine
    from distributed_pytorch_amd.models import VGG11

    ds = synthetic_cifar(2048, 0)
    ld = DeviceLoader(ds, 256, "cuda", sampler=ShardSampler(2048, 1, 0), train=True, seed=1)
    e = VGGEngine("VGG11", "cuda", max_batch=256, impl=impl, lr=0.1)
    e.init_parameters(seed=1)
    for x, t in ld:
        e.forward_backward(x, t)
        e.sgd_step()
        e.finish_step()
    m = VGG11()
    m.load_state_dict(e.state_dict())
    m.eval()
    test = DeviceLoader(synthetic_cifar(512, 1), 256, "cuda", train=False)
    e.begin_eval()
    for x, t in test:
        logits = torch.zeros(x.shape[0], 10, device="cuda")
        e.eval_batch(x, t, logits)
        with torch.no_grad():
            ref = m(x[..., :3].permute(0, 3, 1, 2).cpu())
        torch.cuda.synchronize()
        err = (logits.cpu() - ref).abs().max().item() / ref.abs().max().item()
        assert err < 1e-3, err


@pytest.mark.parametrize("name", ["VGG13", "VGG16", "VGG19"])
def test_other_vgg_depths_step_matches_torch(name):
    """The engine's other reference configs (model.py:3-8 cfg table) on the x3 kernels: one training
    step's loss and a few updated parameters match stock torch (fp32)."""
    from distributed_pytorch_amd.engine import VGGEngine
    from distributed_pytorch_amd.models.vgg import VGG

    torch.manual_seed(3)
    ref = VGG(name)
    e = VGGEngine(name, "cuda", max_batch=16, impl="x3", lr=0.05)
    e.load_state_dict(ref.state_dict())
    before = {k: v.clone() for k, v in ref.state_dict().items()}
    g = torch.Generator().manual_seed(5)
    x = torch.randn(16, 3, 32, 32, generator=g)
    t = torch.randint(0, 10, (16,), generator=g)
    x4 = torch.zeros(16, 32, 32, 4)
    x4[..., :3] = x.permute(0, 2, 3, 1)
    e.forward_backward(x4.cuda(), t.cuda())
    e.sgd_step()
    e.finish_step()
    opt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    loss = F.cross_entropy(ref(x), t)
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    assert abs(float(e.loss.item()) - float(loss)) < 1e-4 * max(1.0, float(loss))
    sd = e.state_dict()
    for k, v in ref.state_dict().items():
        if v.is_floating_point() and "running" not in k:
            du, dr = sd[k] - before[k], v - before[k]  # the SGD updates (fp32 sums through up to 16 BNs)
            if dr.norm().item() < 1e-5:
                continue  # conv biases: analytic gradient 0, the update is rounding noise + weight decay
            assert (du - dr).norm().item() <= 1e-2 * dr.norm().item(), k  # deep + batch 16: ill-conditioned


@pytest.mark.parametrize("impl", ["x3", "bf16"])
def test_wgrad_stream_matches_single_stream(monkeypatch, impl):
    """Weight gradients on the second HIP stream train bit-identically to the single-stream
    schedule, both with per-layer events and with the kernel-start signals (the default,
    signal.hip): the cross-stream ordering loses no dependency."""
    from distributed_pytorch_amd.engine import VGGEngine

    g = torch.Generator().manual_seed(5)
    xs = [torch.randn(64, 32, 32, 4, generator=g) for _ in range(3)]
    ts = [torch.randint(0, 10, (64,), generator=g) for _ in range(3)]
    outs = []
    for stream, ksig in (("0", "0"), ("1", "0"), ("1", "1")):
        monkeypatch.setenv("DPA_WGRAD_STREAM", stream)
        monkeypatch.setenv("DPA_KSIGNAL", ksig)
        e = VGGEngine("VGG11", "cuda", max_batch=64, impl=impl, lr=0.01)
        e.init_parameters(seed=3)
        assert (e.wstream is not None) == (stream == "1")
        assert e.ksignal == (stream == "1" and ksig == "1")
        for x, t in zip(xs, ts):
            x = x.cuda()
            x[..., 3] = 0
            e.forward_backward(x, t.cuda())
            e.sgd_step()
            e.finish_step()
        torch.cuda.synchronize()
        e.check_signals()
        if e.ksignal:
            assert e.ksig[1:].tolist() == [3] * (len(e.spec.convs) - 1)  # every side layer signalled 3 steps
            assert e.bsig.tolist() == [3] * len(e.spec.convs)  # ... and every BN backward
        outs.append(e.params.flat.clone())
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("impl", ["x3", "bf16"])
def test_graphed_step_matches_eager(impl):
    """The captured HIP-graph step (both streams, fused SGD) replays to bit-identical parameters,
    momentum and loss as the eager step, across several replays."""
    from distributed_pytorch_amd.engine import VGGEngine
    from distributed_pytorch_amd.graph_step import GraphedStep
    from distributed_pytorch_amd.parallel import NullComm, make_sync

    g = torch.Generator().manual_seed(21)
    batches = [(torch.randn(32, 32, 32, 4, generator=g), torch.randint(0, 10, (32,), generator=g)) for _ in range(5)]
    outs = []
    for graph in (False, True):
        e = VGGEngine("VGG11", "cuda", max_batch=32, impl=impl, lr=0.02)
        e.init_parameters(seed=4)
        sync = make_sync("ddp", e, NullComm())
        gs = GraphedStep(e, sync, warmup=2) if graph else None
        xb = torch.empty(32, 32, 32, 4, device="cuda")
        tb = torch.empty(32, dtype=torch.int64, device="cuda")
        losses = []
        for x, t in batches:
            xb.copy_(x)
            xb[..., 3] = 0
            tb.copy_(t)
            if gs is not None:
                gs.run(xb, tb)
            else:
                sync.begin_step()
                e.forward_backward(xb, tb, grad_ready=sync.grad_ready, pre_forward=sync.pre_forward,
                                   params_free=sync.params_free)
                sync.update(sync.finish())
                e.finish_step()
            losses.append(e.loss.clone())
        torch.cuda.synchronize()
        if gs is not None:
            assert gs.replays == 3 and gs.graph is not None
        outs.append((e.params.flat.clone(), e.mom.flat.clone(), torch.stack(losses)))
    for a_, b_ in zip(outs[0], outs[1]):
        assert torch.equal(a_, b_)


def test_fused_head_matches_separate_bn_apply(monkeypatch):
    """The last layer's BN + ReLU + 2x2 max-pool computed inside the classifier kernel (fc_ce.hip
    BnIn) instead of by bn_apply: same operations in the same order, so training is bit-identical."""
    from distributed_pytorch_amd.engine import VGGEngine

    g = torch.Generator().manual_seed(13)
    xs = [torch.randn(64, 32, 32, 4, generator=g) for _ in range(2)]
    ts = [torch.randint(0, 10, (64,), generator=g) for _ in range(2)]
    outs = []
    for fused in ("0", "1"):
        monkeypatch.setenv("DPA_FUSED_HEAD", fused)
        e = VGGEngine("VGG11", "cuda", max_batch=64, impl="x3", lr=0.05)
        assert e.fused_head == (fused == "1")
        e.init_parameters(seed=6)
        losses = []
        for x, t in zip(xs, ts):
            x = x.cuda()
            x[..., 3] = 0
            e.forward_backward(x, t.cuda())
            e.sgd_step()
            e.finish_step()
            losses.append(e.loss.clone())
        torch.cuda.synchronize()
        outs.append((e.params.flat.clone(), e.a[-1].clone(), torch.cat(losses)))
    for a_, b_ in zip(*outs):
        assert torch.equal(a_, b_)
