"""BatchNorm2d (+ReLU, +2x2 max-pool) kernels against torch's own autograd in fp64.

The oracle is ``F.batch_norm(training=True)`` -> ``relu`` -> ``max_pool2d(2, 2)`` of the reference
layer chain (/root/reference/model.py:16,24,25) run in float64 on the CPU, forward and backward —
not the framework's own CPU mirror.  Both BN paths are checked: the three-kernel path (bn.hip:
statistics -> finalize -> apply; reduce -> finalize -> apply) and the one-launch path
(bn_fused.hip) the VGG engine uses for its small layers.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

EPS, MOM = 1e-5, 0.1


def _C():
    from distributed_pytorch_amd import _ext

    return _ext.require()


def close(a, b, tol, what=""):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    d = (a - b).abs().max().item()
    s = b.abs().max().clamp_min(1e-6).item()
    assert d <= tol * s, f"{what}: max abs diff {d} vs scale {s}"


def oracle(z, gamma, beta, bias, rm, rv, pool, gout=None):
    """fp64 torch reference of the layer tail (conv bias folded in as the kernels do: z excludes it).
    Returns dict with a (NHWC), mean/invstd of z, updated running stats and, given gout (NHWC), the
    gradients dz (NHWC), dgamma, dbeta, dbias."""
    x = (z.double().permute(0, 3, 1, 2) + bias.double().view(1, -1, 1, 1)).detach().requires_grad_(True)
    gm = gamma.double().clone().requires_grad_(True)
    bt = beta.double().clone().requires_grad_(True)
    rm_, rv_ = rm.double().clone(), rv.double().clone()
    y = F.relu(F.batch_norm(x, rm_, rv_, gm, bt, training=True, momentum=MOM, eps=EPS))
    if pool:
        y = F.max_pool2d(y, 2, 2)
    out = {"a": y.detach().permute(0, 2, 3, 1), "rm": rm_, "rv": rv_}
    zz = z.double().reshape(-1, z.shape[-1])
    out["mean"] = zz.mean(0)
    out["invstd"] = torch.rsqrt(zz.var(0, unbiased=False) + EPS)
    if gout is not None:
        y.backward(gout.double().permute(0, 3, 1, 2))
        out["dz"] = x.grad.permute(0, 2, 3, 1)
        out["dgamma"], out["dbeta"] = gm.grad, bt.grad
        out["dbias"] = x.grad.sum((0, 2, 3))
    return out


def _inputs(shape, seed):
    """z on a grid of 0.25-spaced levels and beta placing every channel's ReLU threshold half-way
    between two levels: the fp32 kernels and the fp64 oracle then route every 2x2 max and every
    ReLU mask the same way (equal values tie exactly in both, first max wins; distinct values are
    >= 0.25 apart, and no value sits within ~0.01 of the threshold)."""
    N, H, W, C, pool = shape
    g = torch.Generator().manual_seed(seed)
    z = torch.randint(-40, 41, (N, H, W, C), generator=g).float() * 0.25 + 1.5
    gamma, bias = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g)
    zz = z.double().reshape(-1, C)
    thr = torch.randint(-12, 13, (C,), generator=g).double() * 0.25 + 1.5 + 0.125
    beta = (-gamma.double() * (thr - zz.mean(0)) * torch.rsqrt(zz.var(0, unbiased=False) + EPS)).float()
    rm, rv = torch.randn(C, generator=g), torch.rand(C, generator=g) + 0.5
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    gout = torch.randn(N, Ho, Wo, C, generator=g)
    if pool:  # exact ties at a window's positive maximum: no gradient (torch's tie routing is machine-dependent)
        zz4 = z.double()
        y = torch.relu((zz4 - zz.mean(0)) * torch.rsqrt(zz.var(0, unbiased=False) + EPS) * gamma.double() + beta.double())
        win = y.reshape(N, Ho, 2, Wo, 2, C).permute(0, 1, 3, 5, 2, 4).reshape(N, Ho, Wo, C, 4)
        top = win.sort(-1, descending=True).values
        gout[(top[..., 0] == top[..., 1]) & (top[..., 0] > 0)] = 0.0
    return g, z, gamma, beta, bias, rm, rv, gout


def _planes_sum(p):
    return p.float().sum(0)


BN_SHAPES = [(4, 32, 32, 64, True), (4, 16, 16, 128, True), (8, 8, 8, 256, False), (16, 2, 2, 512, True),
             (3, 6, 6, 16, False), (2, 4, 4, 256, True)]


@pytest.mark.parametrize("shape", BN_SHAPES)
def test_bn_three_kernel_forward(shape):
    C_ = _C()
    N, H, W, C, pool = shape
    g, z, gamma, beta, bias, rm, rv, _ = _inputs(shape, 0)
    ref = oracle(z, gamma, beta, bias, rm, rv, pool)
    d = lambda t: t.cuda()
    sl = torch.randn(3, *z.shape, generator=g)  # split-K path: z arrives as 3 slabs that sum to it
    sl[2] = z - sl[0] - sl[1]
    zd = torch.empty(z.shape, device="cuda")
    part = torch.zeros(C_.bn_part_floats(N * H * W, C, False), device="cuda")
    mean, invstd, scale, shift = (torch.zeros(C, device="cuda") for _ in range(4))
    rm_d, rv_d, nbt_d = d(rm), d(rv), torch.zeros(1, dtype=torch.int64, device="cuda")
    C_.bn_fwd_stats(d(sl.reshape(-1)), 3, zd, part, d(gamma), d(beta), d(bias), rm_d, rv_d, nbt_d, mean, invstd,
                    scale, shift, MOM, EPS)
    a = torch.empty(ref["a"].shape, device="cuda")
    C_.bn_apply(zd, a, scale, shift, pool)
    torch.cuda.synchronize()
    close(zd, z, 1e-5, "z")
    close(a, ref["a"], 1e-5, "a")
    close(mean, ref["mean"], 1e-5, "mean")
    close(invstd, ref["invstd"], 1e-5, "invstd")
    close(rm_d, ref["rm"], 1e-5, "running_mean")
    close(rv_d, ref["rv"], 1e-5, "running_var")
    assert int(nbt_d.item()) == 1


def _h2_act(a):
    """Activation value of fp16-pair planes (fixed scale 16)."""
    return (a[0].float() + a[1].float()) / 16.0


@pytest.mark.parametrize("shape", BN_SHAPES)
def test_bn_apply_fp16_pair_planes(shape):
    """bn_apply into fp16-pair activation planes (impl "h2"), pooled and not: the pair holds
    a * 16 to 2^-21 relative (vs the fp32 apply of the same z, scale and shift)."""
    C_ = _C()
    N, H, W, C, pool = shape
    g = torch.Generator().manual_seed(9)
    z = torch.randn(N, H, W, C, generator=g).cuda()
    scale = (torch.rand(C, generator=g) + 0.5).cuda()
    shift = torch.randn(C, generator=g).cuda() * 0.1
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    a32 = torch.empty(N, Ho, Wo, C, device="cuda")
    C_.bn_apply(z, a32, scale, shift, pool)
    a2 = torch.empty(2, N, Ho, Wo, C, device="cuda", dtype=torch.float16)
    C_.bn_apply(z, a2, scale, shift, pool)
    torch.cuda.synchronize()
    err = (_h2_act(a2).double() - a32.double()).abs()
    tol = torch.maximum(a32.double().abs() * 2.0 ** -21, torch.full_like(err, 2.0 ** -29))
    assert (err <= tol).all(), (err / tol).max().item()


@pytest.mark.parametrize("shape", BN_SHAPES + [(256, 16, 16, 128, True), (256, 8, 8, 256, False)])
@pytest.mark.parametrize("nsplit", [1, 2])
def test_bn_three_kernel_backward(shape, nsplit):
    C_ = _C()
    N, H, W, C, pool = shape
    g, z, gamma, beta, bias, rm, rv, gout = _inputs(shape, 1)
    ref = oracle(z, gamma, beta, bias, rm, rv, pool, gout)
    mean, invstd = ref["mean"].float(), ref["invstd"].float()
    scale, shift = gamma * invstd, beta - mean * gamma * invstd
    d = lambda t: t.cuda()
    Ho, Wo = gout.shape[1:3]
    part = torch.zeros(C_.bn_part_floats(N * Ho * Wo, C, True), device="cuda")
    coef = torch.empty(4 * C, device="cuda")
    out = [torch.zeros(C, device="cuda") for _ in range(3)]
    dz = torch.empty(z.shape, device="cuda")
    if nsplit == 1:
        src = gbuf = d(gout)
    else:
        half = torch.randn(gout.shape, generator=g)
        src, gbuf = d(torch.stack([half, gout - half]).reshape(-1)), torch.empty(gout.shape, device="cuda")
    C_.bn_bwd(src, nsplit, gbuf, d(z), d(scale), d(shift), d(mean), d(invstd), d(gamma), part, coef, out[0],
              out[1], out[2], dz, pool)
    torch.cuda.synchronize()
    close(gbuf, gout, 1e-5, "g")
    close(dz, ref["dz"], 2e-5, "dz")
    close(out[0], ref["dgamma"], 2e-5, "dgamma")
    close(out[1], ref["dbeta"], 2e-5, "dbeta")
    assert out[2].abs().max().item() < 1e-3 * ref["dbeta"].abs().max().item() + 1e-4  # dbias ~ 0


@pytest.mark.parametrize("shape", BN_SHAPES + [(256, 8, 8, 256, False)])
@pytest.mark.parametrize("nsplit", [1, 2])
def test_bn_backward_fp16_pair_planes(shape, nsplit):
    """fp16-pair dz planes (impl "h2"): the reduce pass tracks max|dy| and max|z|, the finalize writes
    the bound |k1| max|dy| + |k2| max|z| + |k3| (maximised over the channels) into the bound word,
    and the apply pass stores the pair of dz * s with s = 2^(14 - e), bound < 2^e.  The pair must
    hold dz to 2^-21 relative of the tensor's scale (the fp32 apply's own dz, bitwise the same
    statistics), the bound must cover every |dz|, and |dz s| stay below 2^14."""
    import math

    C_ = _C()
    N, H, W, C, pool = shape
    g, z, gamma, beta, bias, rm, rv, gout = _inputs(shape, 1)
    ref = oracle(z, gamma, beta, bias, rm, rv, pool, gout)
    mean, invstd = ref["mean"].float(), ref["invstd"].float()
    scale, shift = gamma * invstd, beta - mean * gamma * invstd
    d = lambda t: t.cuda()
    Ho, Wo = gout.shape[1:3]
    part = torch.zeros(C_.bn_part_floats(N * Ho * Wo, C, True), device="cuda")
    outs = []
    for kind in ("fp32", "h2"):
        coef = torch.empty(4 * C, device="cuda")
        o = [torch.zeros(C, device="cuda") for _ in range(3)]
        dz = (torch.empty(z.shape, device="cuda") if kind == "fp32"
              else torch.empty((2,) + tuple(z.shape), device="cuda", dtype=torch.float16))
        bound = torch.full((1,), -1, dtype=torch.int32, device="cuda")  # the reduce re-arms it
        if nsplit == 1:
            src = gbuf = d(gout)
        else:
            half = torch.randn(gout.shape, generator=torch.Generator().manual_seed(5))
            src, gbuf = d(torch.stack([half, gout - half]).reshape(-1)), torch.empty(gout.shape, device="cuda")
        C_.bn_bwd(src, nsplit, gbuf, d(z), d(scale), d(shift), d(mean), d(invstd), d(gamma), part, coef, o[0], o[1],
                  o[2], dz, pool, **({"bound": bound} if kind == "h2" else {}))
        torch.cuda.synchronize()
        outs.append((dz, coef, o, bound))
    dz32, coef32, o32, _ = outs[0]
    dzh, coefh, oh, bound = outs[1]
    assert torch.equal(coef32, coefh) and all(torch.equal(a_, b_) for a_, b_ in zip(o32, oh))
    B = float(bound.view(torch.float32).item())
    s = 2.0 ** (14 - math.frexp(B)[1])
    rec = (dzh[0].float().double() + dzh[1].float().double()) / s
    assert B >= dz32.abs().max().item() > 0
    assert dzh.float().abs().max().item() * 1.0 <= 2.0 ** 14 + 1
    assert (rec - dz32.double()).abs().max().item() <= 2.0 ** -21 * dz32.abs().max().item()


# ---------------------------------------------------------------- one-launch BN (bn_fused.hip)
# VGG-11's tail at batch 256 (layers 2-7) and small odd batches; rmax 64 = the engine default
FUSED_SHAPES = [(256, 8, 8, 256, False), (256, 8, 8, 256, True), (256, 4, 4, 512, False), (256, 4, 4, 512, True),
                (256, 2, 2, 512, False), (256, 2, 2, 512, True), (16, 2, 2, 512, True), (32, 4, 4, 64, True),
                (64, 2, 2, 96, False)]


def _fused_ws(C_, shape, bwd, rmax):
    N, H, W, C, pool = shape
    Mo = N * ((H // 2) * (W // 2) if pool else H * W)
    geo = C_.bn_fused_geo(Mo, C, pool, bwd, rmax)
    if geo is None:
        return None
    pf, cw, _ = geo
    return torch.zeros(pf, device="cuda"), torch.zeros(cw, dtype=torch.int32, device="cuda")


@pytest.mark.parametrize("shape", FUSED_SHAPES)
@pytest.mark.parametrize("nsplit", [1, 3])
@pytest.mark.parametrize("out_kind", ["planes", "fp32", "none", "h2"])
def test_bn_fused_forward(shape, nsplit, out_kind):
    C_ = _C()
    N, H, W, C, pool = shape
    ws = _fused_ws(C_, shape, False, 128)
    assert ws is not None, "no one-launch geometry for a VGG shape"
    part, cnt = ws
    g, z, gamma, beta, bias, rm, rv, _ = _inputs(shape, 5)
    ref = oracle(z, gamma, beta, bias, rm, rv, pool)
    d = lambda t: t.cuda()
    if nsplit == 1:
        src = d(z)
        zd = src
    else:
        sl = torch.randn(3, *z.shape, generator=g)
        sl[2] = z - sl[0] - sl[1]
        src, zd = d(sl.reshape(-1)), torch.empty(z.shape, device="cuda")
    outs = []
    for rep in range(2):  # second launch: the slice counters must have reset themselves
        mean, invstd, scale, shift = (torch.zeros(C, device="cuda") for _ in range(4))
        rm_d, rv_d, nbt_d = d(rm), d(rv), torch.zeros(1, dtype=torch.int64, device="cuda")
        tmo = torch.zeros(1, dtype=torch.int32, device="cuda")
        if out_kind == "planes":
            a = torch.empty(3, *ref["a"].shape, device="cuda", dtype=torch.bfloat16)
        elif out_kind == "h2":
            a = torch.empty(2, *ref["a"].shape, device="cuda", dtype=torch.float16)
        elif out_kind == "fp32":
            a = torch.empty(ref["a"].shape, device="cuda")
        else:
            a = None
        C_.bn_fused_fwd(src, nsplit, zd, pool, 128, part, cnt, d(gamma), d(beta), d(bias), rm_d, rv_d, nbt_d, mean,
                        invstd, scale, shift, a, MOM, EPS, tmo, 5_000_000)
        torch.cuda.synchronize()
        assert int(tmo.item()) == 0
        assert int(cnt.abs().sum().item()) == 0, "slice counters not reset"
        close(zd, z, 1e-5, "z")
        close(mean, ref["mean"], 1e-5, "mean")
        close(invstd, ref["invstd"], 1e-5, "invstd")
        close(rm_d, ref["rm"], 1e-5, "running_mean")
        close(rv_d, ref["rv"], 1e-5, "running_var")
        assert int(nbt_d.item()) == 1
        if a is not None:
            close(_planes_sum(a) if out_kind == "planes" else _h2_act(a) if out_kind == "h2" else a, ref["a"], 1e-5,
                  "a")
        outs.append([t.clone() for t in (mean, invstd, scale, shift) + ((a,) if a is not None else ())])
    for x, y in zip(*outs):
        assert torch.equal(x, y), "one-launch BN forward is not deterministic"


@pytest.mark.parametrize("shape", FUSED_SHAPES)
@pytest.mark.parametrize("nsplit", [1, 2])
@pytest.mark.parametrize("out_kind", ["planes", "fp32"])
def test_bn_fused_backward(shape, nsplit, out_kind):
    C_ = _C()
    N, H, W, C, pool = shape
    ws = _fused_ws(C_, shape, True, 128)
    assert ws is not None, "no one-launch geometry for a VGG shape"
    part, cnt = ws
    g, z, gamma, beta, bias, rm, rv, gout = _inputs(shape, 6)
    ref = oracle(z, gamma, beta, bias, rm, rv, pool, gout)
    mean, invstd = ref["mean"].float(), ref["invstd"].float()
    scale, shift = gamma * invstd, beta - mean * gamma * invstd
    d = lambda t: t.cuda()
    if nsplit == 1:
        src = d(gout)
    else:
        half = torch.randn(gout.shape, generator=g)
        src = d(torch.stack([half, gout - half]).reshape(-1))
    sig = torch.zeros(1, dtype=torch.int32, device="cuda")
    outs = []
    for rep in range(2):
        dg, db, dbias = (torch.zeros(C, device="cuda") for _ in range(3))
        dz = (torch.empty(3, *z.shape, device="cuda", dtype=torch.bfloat16) if out_kind == "planes"
              else torch.empty(z.shape, device="cuda"))
        tmo = torch.zeros(1, dtype=torch.int32, device="cuda")
        C_.bn_fused_bwd(src, nsplit, d(z), pool, 128, part, cnt, d(scale), d(shift), d(mean), d(invstd), d(gamma), dg,
                        db, dbias, dz, tmo, 5_000_000, sig=sig, sig_val=rep + 7)
        torch.cuda.synchronize()
        assert int(tmo.item()) == 0
        assert int(cnt.abs().sum().item()) == 0, "slice counters not reset"
        assert int(sig.item()) == rep + 7, "kernel-start signal not raised"
        close(_planes_sum(dz) if out_kind == "planes" else dz, ref["dz"], 2e-5, "dz")
        close(dg, ref["dgamma"], 2e-5, "dgamma")
        close(db, ref["dbeta"], 2e-5, "dbeta")
        assert dbias.abs().max().item() < 1e-3 * ref["dbeta"].abs().max().item() + 1e-4  # dbias ~ 0
        outs.append([t.clone() for t in (dg, db, dbias, dz)])
    for x, y in zip(*outs):
        assert torch.equal(x, y), "one-launch BN backward is not deterministic"


def test_bn_fused_geometry_limits():
    """The geometry query refuses shapes whose row blocks per slice exceed rmax or whose channels
    are not a multiple of 32, and every VGG-11 tail layer at batch 256 fits rmax 64 forward."""
    C_ = _C()
    assert C_.bn_fused_geo(256 * 64, 24, False, False, 64) is None
    assert C_.bn_fused_geo(1 << 20, 64, False, False, 64) is None
    for mo, c, pool in ((256 * 4, 512, True), (256 * 16, 512, False), (256 * 4, 512, False), (256, 512, True),
                        (256 * 16, 256, True), (256 * 64, 256, False)):
        geo = C_.bn_fused_geo(mo, c, pool, False, 64)
        assert geo is not None and geo[2] <= 512, (mo, c, pool, geo)


def test_bn_fused_residency_guard_falls_back(monkeypatch):
    """a one-launch BN grid that could exceed the co-resident capacity is refused
    by the geometry query (DPA_BN_FUSED_CAP pretends a small chip), and the engine then runs the
    three-kernel BN for every layer; the step still trains and matches the default engine."""
    from distributed_pytorch_amd.engine import VGGEngine

    C_ = _C()
    assert C_.bn_fused_geo(256 * 4, 512, True, False, 64) is not None
    monkeypatch.setenv("DPA_BN_FUSED_CAP", "1")
    assert C_.bn_fused_geo(256 * 4, 512, True, False, 64) is None
    torch.manual_seed(0)
    x = torch.zeros(64, 32, 32, 4, device="cuda")
    x[..., :3] = torch.randn(64, 32, 32, 3, device="cuda")
    t = torch.randint(0, 10, (64,), device="cuda")
    res = []
    for cap in ("1", None):
        if cap is None:
            monkeypatch.delenv("DPA_BN_FUSED_CAP")
        eng = VGGEngine("VGG11", "cuda", max_batch=64, impl="x3")
        eng.init_parameters(seed=1)
        fused = [eng._fused(i, 64, b) for i in range(8) for b in (False, True)]
        assert any(fused) == (cap is None), fused
        loss = float(eng.forward_backward(x, t).item())
        torch.cuda.synchronize()
        eng.check_signals()
        res.append((loss, eng.grads.flat.clone()))
    assert abs(res[0][0] - res[1][0]) <= 1e-4 * abs(res[1][0])
    rel = ((res[0][1] - res[1][1]).norm() / res[1][1].norm()).item()
    assert rel < 1e-3, rel


def test_bn_fused_rendezvous_timeout_sets_flag(monkeypatch):
    """A slice rendezvous that can never complete (test-only phantom arrivals) gives up after its
    own short bound, raises the timeout word and leaves the counters re-armed: no hang."""
    C_ = _C()
    shape = (256, 4, 4, 512, True)
    ws = _fused_ws(C_, shape, False, 64)
    part, cnt = ws
    g, z, gamma, beta, bias, rm, rv, _ = _inputs(shape, 5)
    d = lambda t: t.cuda()
    monkeypatch.setenv("DPA_BN_FUSED_TEST_PHANTOM", "1")
    mean, invstd, scale, shift = (torch.zeros(512, device="cuda") for _ in range(4))
    tmo = torch.zeros(1, dtype=torch.int32, device="cuda")
    zd = d(z)
    C_.bn_fused_fwd(zd, 1, zd, True, 64, part, cnt, d(gamma), d(beta), d(bias), d(rm), d(rv), None, mean, invstd,
                    scale, shift, None, MOM, EPS, tmo, 20_000)
    torch.cuda.synchronize()
    assert int(tmo.item()) == 1
    assert int(cnt.abs().sum().item()) == 0, "slice counters not reset after a timeout"
    monkeypatch.delenv("DPA_BN_FUSED_TEST_PHANTOM")
    tmo.zero_()
    C_.bn_fused_fwd(zd, 1, zd, True, 64, part, cnt, d(gamma), d(beta), d(bias), d(rm), d(rv), None, mean, invstd,
                    scale, shift, None, MOM, EPS, tmo, 2_000_000)
    torch.cuda.synchronize()
    assert int(tmo.item()) == 0
