"""Numerics of every HIP kernel against a plain PyTorch fp32/fp64 reference of the same op.

Shapes: the VGG-11 layer shapes of SURVEY §2.3 (with a reduced batch so the fp64 CPU
reference stays cheap) plus odd shapes exercising masking / split-K / tails.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _C():
    from distributed_pytorch_amd import _ext

    return _ext.require()


def rel_err(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


CONV_SHAPES = [
    # N, H, W, C, K, R, stride, pad
    (8, 32, 32, 4, 64, 3, 1, 1),
    (8, 16, 16, 64, 128, 3, 1, 1),
    (4, 8, 8, 128, 256, 3, 1, 1),
    (4, 4, 4, 256, 512, 3, 1, 1),
    (16, 2, 2, 512, 512, 3, 1, 1),
    (3, 7, 5, 12, 20, 3, 1, 1),
    (2, 9, 9, 8, 16, 3, 2, 1),
    (2, 8, 8, 16, 32, 1, 1, 0),
    (2, 14, 14, 4, 16, 7, 2, 3),
]


CONV_SHAPES += [(128, 4, 4, 32, 64, 3, 1, 1), (64, 2, 2, 64, 32, 3, 1, 1), (128, 8, 8, 32, 32, 3, 1, 1),
                (64, 5, 5, 64, 64, 3, 2, 1)]


@pytest.mark.parametrize("shape", CONV_SHAPES)
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("tile", [0, 1])
@pytest.mark.parametrize("posmajor", [False, True])
def test_conv_fprop(shape, splits, tile, posmajor):
    C = _C()
    N, H, W, Cin, K, R, st, pd = shape
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(K, Cin, R, R, generator=g) * 0.1
    ref = F.conv2d(x.double(), w.double(), stride=st, padding=pd)  # N K P Q
    xd = x.permute(0, 2, 3, 1).contiguous().cuda()
    wd = w.permute(0, 2, 3, 1).contiguous().cuda()
    P, Q = ref.shape[2], ref.shape[3]
    out = torch.empty(N, P, Q, K, device="cuda")
    slab = torch.empty(splits * N * P * Q * K, device="cuda") if splits > 1 else None
    C.conv_fprop(xd, wd, out, slab, st, pd, splits, tile, False, True, posmajor)
    torch.cuda.synchronize()
    assert rel_err(out.permute(0, 3, 1, 2), ref) < 1e-5


@pytest.mark.parametrize("shape", CONV_SHAPES)
@pytest.mark.parametrize("splits", [1, 7])
@pytest.mark.parametrize("tile", [0, 1])
@pytest.mark.parametrize("posmajor", [False, True])
def test_conv_wgrad(shape, splits, tile, posmajor):
    C = _C()
    N, H, W, Cin, K, R, st, pd = shape
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64, requires_grad=False)
    w = (torch.randn(K, Cin, R, R, generator=g, dtype=torch.float64) * 0.1).requires_grad_(True)
    y = F.conv2d(x, w, stride=st, padding=pd)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (gw,) = torch.autograd.grad(y, w, dy)
    xd = x.float().permute(0, 2, 3, 1).contiguous().cuda()
    dzd = dy.float().permute(0, 2, 3, 1).contiguous().cuda()
    dw = torch.empty(K, R, R, Cin, device="cuda")
    slab = torch.empty(splits * K * R * R * Cin, device="cuda") if splits > 1 else None
    C.conv_wgrad(xd, dzd, dw, slab, st, pd, splits, tile, posmajor)
    torch.cuda.synchronize()
    assert rel_err(dw.permute(0, 3, 1, 2), gw) < 1e-5


@pytest.mark.parametrize("shape", [s for s in CONV_SHAPES if s[6] == 1 and 2 * s[7] == s[5] - 1])
def test_conv_dgrad_via_flip(shape):
    C = _C()
    N, H, W, Cin, K, R, st, pd = shape
    g = torch.Generator().manual_seed(2)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64).requires_grad_(True)
    w = torch.randn(K, Cin, R, R, generator=g, dtype=torch.float64) * 0.1
    y = F.conv2d(x, w, stride=st, padding=pd)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (gx,) = torch.autograd.grad(y, x, dy)
    wk = w.float().permute(0, 2, 3, 1).contiguous().cuda()
    wflip = torch.empty(Cin, R, R, K, device="cuda")
    C.wflip(wk, wflip)
    dzd = dy.float().permute(0, 2, 3, 1).contiguous().cuda()
    dx = torch.empty(N, H, W, Cin, device="cuda")
    C.conv_fprop(dzd, wflip, dx, None, 1, pd, 1, 0)
    torch.cuda.synchronize()
    assert rel_err(dx.permute(0, 3, 1, 2), gx) < 1e-5


@pytest.mark.parametrize("shape", [s for s in CONV_SHAPES if s[6] == 1 and 2 * s[7] == s[5] - 1])
@pytest.mark.parametrize("splits", [1, 4])
@pytest.mark.parametrize("tile", [0, 1])
@pytest.mark.parametrize("posmajor", [False, True])
def test_conv_dgrad_mode(shape, splits, tile, posmajor):
    """dgrad=True reads the original KRSC weights with flipped taps (no transposed copy); with
    reduce=False the split-K slabs must sum to the result."""
    C = _C()
    N, H, W, Cin, K, R, st, pd = shape
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64).requires_grad_(True)
    w = torch.randn(K, Cin, R, R, generator=g, dtype=torch.float64) * 0.1
    y = F.conv2d(x, w, stride=st, padding=pd)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (gx,) = torch.autograd.grad(y, x, dy)
    wk = w.float().permute(0, 2, 3, 1).contiguous().cuda()
    dzd = dy.float().permute(0, 2, 3, 1).contiguous().cuda()
    dx = torch.zeros(N, H, W, Cin, device="cuda")
    eff = C.conv_splits(R * R * K, splits)
    slab = torch.empty(eff * N * H * W * Cin, device="cuda") if eff > 1 else None
    C.conv_fprop(dzd, wk, dx, slab, 1, pd, splits, tile, True, False, posmajor)
    torch.cuda.synchronize()
    res = slab.view(eff, N, H, W, Cin).sum(0) if eff > 1 else dx
    assert rel_err(res.permute(0, 3, 1, 2), gx) < 1e-5


# ----------------------------------------------------------------- bf16-plane (x3) kernels
X3_SHAPES = [
    (8, 16, 16, 64, 128, 3, 1, 1),
    (4, 8, 8, 128, 256, 3, 1, 1),
    (128, 4, 4, 64, 64, 3, 1, 1),
    (128, 2, 2, 32, 64, 3, 1, 1),
    (3, 7, 5, 24, 40, 3, 1, 1),
    (2, 9, 9, 16, 32, 3, 2, 1),
    (2, 8, 8, 16, 32, 1, 1, 0),
    (64, 5, 5, 64, 64, 3, 2, 1),
]


def _planes(t, np_):
    """Operand planes of t: bf16 (np 1 / 3), or np 2 float16 pairs of t * s with s the power of two
    that puts max|t| just below 2^14 (as the engine's scales); s is kept as out._h2s."""
    import math

    C = _C()
    if np_ == 2:
        m = float(t.abs().max())
        s = 2.0 ** (14 - math.frexp(m)[1]) if m > 0 else 1.0
        out = torch.empty((2,) + tuple(t.shape), device="cuda", dtype=torch.float16)
        C.split_planes(t.contiguous().cuda(), out, s)
    else:
        s = 1.0
        out = torch.empty((np_,) + tuple(t.shape), device="cuda", dtype=torch.bfloat16)
        C.split_planes(t.contiguous().cuda(), out)
    out._h2s = s
    return out


def _osc(a, b):
    """conv keywords undoing two fp16-pair operands' scales (empty for bf16 planes)."""
    return {"oscale": 1.0 / (a._h2s * b._h2s)} if a.dtype == torch.float16 else {}


def test_split_planes_exact():
    g = torch.Generator().manual_seed(11)
    x = torch.randn(4096, generator=g) * torch.exp(torch.randn(4096, generator=g) * 4)
    p = _planes(x, 3).float().cpu()
    rec = p[0].double() + p[1].double() + p[2].double()
    rel = ((rec - x.double()).abs() / x.double().abs().clamp_min(1e-30)).max().item()
    assert rel < 2 ** -22
    p1 = _planes(x, 1).float().cpu()
    assert torch.equal(p1[0], x.bfloat16().float())


def test_split_planes_fp16_pair_exact():
    """fp16 pairs (impl "h2"): x * s = h0 + h1 to 2^-21 relative, or 2^-25 absolute (in scaled
    units) where the low half is subnormal; the overflow word stays clear."""
    C = _C()
    assert not C.h2_overflow(True)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(4096, generator=g) * torch.exp(torch.randn(4096, generator=g) * 2)
    p = _planes(x, 2)
    s = p._h2s
    rec = (p[0].float().double().cpu() + p[1].float().double().cpu()) / s
    xd = x.double()
    # h1 carries ~11 more bits than h0 until it drops into float16's subnormals (absolute 2^-25)
    tol = torch.maximum(xd.abs() * 2.0 ** -21, torch.full_like(xd, 2.0 ** -25 / s))
    assert ((rec - xd).abs() <= tol).all(), ((rec - xd).abs() / tol).max().item()
    torch.cuda.synchronize()
    assert not C.h2_overflow(False)


def test_fp16_pair_overflow_flag():
    """A split that leaves float16's range raises the overflow word (the engine fails the step)."""
    C = _C()
    C.h2_overflow(True)
    out = torch.empty(2, 64, device="cuda", dtype=torch.float16)
    C.split_planes(torch.full((64,), 300.0, device="cuda"), out, 256.0)  # 76800 > 65504
    torch.cuda.synchronize()
    assert C.h2_overflow(True)
    assert not C.h2_overflow(False)


@pytest.mark.parametrize("shape", X3_SHAPES)
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("tile", list(range(16)))
@pytest.mark.parametrize("posmajor", [False, True])
@pytest.mark.parametrize("np_", [3, 2, 1])
def test_conv_x3_fprop(shape, splits, tile, posmajor, np_):
    C = _C()
    N, H, W, Cin, K, R, st, pd = shape
    g = torch.Generator().manual_seed(12)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(K, Cin, R, R, generator=g) * 0.1
    ref = F.conv2d(x.double(), w.double(), stride=st, padding=pd)
    P, Q = ref.shape[2], ref.shape[3]
    x3 = _planes(x.permute(0, 2, 3, 1), np_)
    w3 = _planes(w.permute(0, 2, 3, 1), np_)
    out = torch.empty(N, P, Q, K, device="cuda")
    slab = torch.empty(splits * N * P * Q * K, device="cuda") if splits > 1 else None
    C.conv_x3_fprop(x3, w3, out, slab, st, pd, splits, tile, True, posmajor, **_osc(x3, w3))
    torch.cuda.synchronize()
    assert rel_err(out.permute(0, 3, 1, 2), ref) < (1e-5 if np_ in (2, 3) else 2e-2)


X3_DGRAD_SHAPES = X3_SHAPES + [
    (2, 16, 16, 8, 64, 1, 2, 0),     # ResNet downsample 1x1/s2
    (2, 20, 20, 8, 64, 7, 2, 3),     # ResNet stem 7x7/s2
    (4, 14, 14, 64, 64, 3, 2, 1),    # ResNet 3x3/s2
]


@pytest.mark.parametrize("shape", X3_DGRAD_SHAPES)
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("tile", [0, 1, 5, 6, 7, 8, 11, 12, 14, 15])
@pytest.mark.parametrize("posmajor", [False, True])
@pytest.mark.parametrize("np_", [3, 2, 1])
def test_conv_x3_dgrad(shape, splits, tile, posmajor, np_):
    """Data gradient straight from the forward weight planes (transposed in-LDS reads), including
    strided convs (input dilation)."""
    C = _C()
    N, H, W, Cin, K, R, st, pd = shape
    g = torch.Generator().manual_seed(13)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64).requires_grad_(True)
    w = torch.randn(K, Cin, R, R, generator=g, dtype=torch.float64) * 0.1
    y = F.conv2d(x, w, stride=st, padding=pd)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (gx,) = torch.autograd.grad(y, x, dy)
    w3 = _planes(w.float().permute(0, 2, 3, 1), np_)
    dz3 = _planes(dy.float().permute(0, 2, 3, 1), np_)
    dx = torch.empty(N, H, W, Cin, device="cuda")
    slab = torch.empty(splits * N * H * W * Cin, device="cuda") if splits > 1 else None
    C.conv_x3_dgrad(dz3, w3, dx, slab, st, pd, splits, tile, True, posmajor, **_osc(dz3, w3))
    torch.cuda.synchronize()
    assert rel_err(dx.permute(0, 3, 1, 2), gx) < (1e-5 if np_ in (2, 3) else 2e-2)


@pytest.mark.parametrize("shape", [(4, 16, 16, 32, 64, 1, 2, 0), (4, 14, 14, 32, 64, 3, 2, 1),
                                   (2, 20, 20, 8, 64, 7, 2, 3), (8, 8, 8, 64, 128, 1, 2, 0)])
@pytest.mark.parametrize("phase", ["0", "1"])
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("tile", [5, 10, 14])
@pytest.mark.parametrize("np_", [3, 2, 1])
def test_conv_x3_dgrad_stride2_phases(monkeypatch, shape, phase, splits, tile, np_):
    """Stride-2 data gradient, phase-decomposed (DPA_DGRAD_PHASE=1: one sub-filter gather per
    output phase, zero-tap phases stored as zeros) and in the dilated form (=0), both against fp64
    autograd; bf16 output (one plane) too."""
    monkeypatch.setenv("DPA_DGRAD_PHASE", phase)
    C = _C()
    N, H, W, Cin, K, R, st, pd = shape
    g = torch.Generator().manual_seed(31)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64).requires_grad_(True)
    w = torch.randn(K, Cin, R, R, generator=g, dtype=torch.float64) * 0.1
    y = F.conv2d(x, w, stride=st, padding=pd)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (gx,) = torch.autograd.grad(y, x, dy)
    dt = torch.bfloat16 if (np_ == 1 and splits == 1) else torch.float32
    dx = torch.full((N, H, W, Cin), float("nan"), device="cuda", dtype=dt)  # every element is written
    slab = torch.empty(splits * N * H * W * Cin, device="cuda") if splits > 1 else None
    dz3, w3 = _planes(dy.float().permute(0, 2, 3, 1), np_), _planes(w.float().permute(0, 2, 3, 1), np_)
    C.conv_x3_dgrad(dz3, w3, dx, slab, st, pd, splits, tile, True, False, **_osc(dz3, w3))
    torch.cuda.synchronize()
    assert torch.isfinite(dx.float()).all()
    assert rel_err(dx.float().permute(0, 3, 1, 2), gx) < (1e-5 if np_ in (2, 3) else 2e-2)


def test_conv_x3_planes_as_arena_views():
    """Weight planes may be strided views of one plane arena (the engine's layout)."""
    C = _C()
    g = torch.Generator().manual_seed(15)
    x = torch.randn(4, 32, 8, 8, generator=g)
    w = torch.randn(64, 32, 3, 3, generator=g) * 0.1
    ref = F.conv2d(x.double(), w.double(), padding=1)
    arena = torch.zeros(3, 1000 + w.numel() + 64, device="cuda", dtype=torch.bfloat16)
    wv = arena[:, 1024:1024 + w.numel()].view(3, 64, 3, 3, 32)
    wv.copy_(_planes(w.permute(0, 2, 3, 1), 3))
    out = torch.empty(4, 8, 8, 64, device="cuda")
    C.conv_x3_fprop(_planes(x.permute(0, 2, 3, 1), 3), wv, out, None, 1, 1, 1, 0, True, False)
    torch.cuda.synchronize()
    assert rel_err(out.permute(0, 3, 1, 2), ref) < 1e-5


@pytest.mark.parametrize("shape", X3_SHAPES)
@pytest.mark.parametrize("splits", [1, 7])
@pytest.mark.parametrize("tile", list(range(16)))
@pytest.mark.parametrize("posmajor", [False, True])
@pytest.mark.parametrize("np_", [3, 2, 1])
def test_conv_x3_wgrad(shape, splits, tile, posmajor, np_):
    C = _C()
    N, H, W, Cin, K, R, st, pd = shape
    g = torch.Generator().manual_seed(14)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64)
    w = (torch.randn(K, Cin, R, R, generator=g, dtype=torch.float64) * 0.1).requires_grad_(True)
    y = F.conv2d(x, w, stride=st, padding=pd)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (gw,) = torch.autograd.grad(y, w, dy)
    x3 = _planes(x.float().permute(0, 2, 3, 1), np_)
    dz3 = _planes(dy.float().permute(0, 2, 3, 1), np_)
    dw = torch.empty(K, R, R, Cin, device="cuda")
    slab = torch.empty(splits * K * R * R * Cin, device="cuda") if splits > 1 else None
    C.conv_x3_wgrad(x3, dz3, dw, slab, st, pd, splits, tile, posmajor, **_osc(x3, dz3))
    torch.cuda.synchronize()
    assert rel_err(dw.permute(0, 3, 1, 2), gw) < (1e-5 if np_ in (2, 3) else 2e-2)


def test_x3_accuracy_matches_fp32_mfma():
    """The bf16x6 plane path must be as accurate as the exact-fp32 MFMA path (both vs fp64):
    this is what licenses reporting it as fp32 compute."""
    C = _C()
    N, H, Cin, K = 64, 8, 256, 256
    g = torch.Generator().manual_seed(21)
    x = torch.randn(N, Cin, H, H, generator=g)
    w = torch.randn(K, Cin, 3, 3, generator=g) * 0.05
    ref = F.conv2d(x.double(), w.double(), padding=1)
    xd, wd = x.permute(0, 2, 3, 1).contiguous().cuda(), w.permute(0, 2, 3, 1).contiguous().cuda()
    o32 = torch.empty(N, H, H, K, device="cuda")
    C.conv_fprop(xd, wd, o32, None, 1, 1, 1, 0)
    o3 = torch.empty(N, H, H, K, device="cuda")
    C.conv_x3_fprop(_planes(xd, 3), _planes(wd, 3), o3, None, 1, 1, 1, 5, True, False)
    o1 = torch.empty(N, H, H, K, device="cuda")
    C.conv_x3_fprop(_planes(xd, 1), _planes(wd, 1), o1, None, 1, 1, 1, 5, True, False)
    torch.cuda.synchronize()
    r = ref.permute(0, 2, 3, 1)
    e32 = (o32.double().cpu() - r).abs().max().item()
    e3 = (o3.double().cpu() - r).abs().max().item()
    e1 = (o1.double().cpu() - r).abs().max().item()
    assert e3 <= 2.0 * e32 + 1e-12, (e3, e32)
    assert e1 > 20 * e3  # and the plain bf16 path really is lower precision


@pytest.mark.parametrize("np_", [1, 3])
def test_pad_split8(np_):
    C = _C()
    g = torch.Generator().manual_seed(16)
    x = torch.randn(3, 5, 7, 4, generator=g)
    x[..., 3] = 0
    out = torch.full((np_, 3, 5, 7, 8), 7.0, device="cuda", dtype=torch.bfloat16)
    C.pad_split8(x.cuda(), out)
    torch.cuda.synchronize()
    ref = torch.zeros(3, 5, 7, 8)
    ref[..., :4] = x
    assert torch.equal(out.cpu(), _planes(ref, np_).cpu())


# ----------------------------------------------------------------- halo-staged 3x3 kernels
HALO_SHAPES = [
    # N, H, W, C, K   (3x3, stride 1, pad 1)
    (2, 16, 16, 64, 128),
    (5, 8, 8, 128, 256),    # the last 256-pixel block is partial
    (19, 4, 4, 32, 64),     # blocks span many images
    (3, 2, 2, 64, 32),
    (1, 32, 32, 32, 48),    # blocks are bands of rows; 48 output channels (partial column tile)
    (2, 7, 7, 32, 16),      # ResNet-style odd maps: blocks straddle image boundaries
    (1, 56, 56, 16, 16),    # rows of 56 pixels (fits the 256-pixel tiles only)
    (3, 16, 16, 128, 64),   # VGG layer-1-like data gradient into 64 channels (tiles 20/21)
    (2, 8, 8, 64, 96),      # 96 output channels: one full and one partial 64-column tile
    (2, 12, 12, 192, 128),  # three 64-channel chunks (tiles 22/23), partial 256-pixel block
    (1, 28, 28, 64, 64),    # rows of 28 pixels: 64-channel chunks with one plane only (NP 2 needs <= 16)
]


def _halo_ok(kind, tile, w, cred, cout, np_=2):
    from distributed_pytorch_amd.engine import halo_ok

    return halo_ok(kind, tile, w, cred, cout, np_)


@pytest.mark.parametrize("shape", HALO_SHAPES)
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("tile", [16, 17, 18, 19, 20, 21, 22, 23])
@pytest.mark.parametrize("np_", [3, 2, 1])
@pytest.mark.parametrize("dgrad", [False, True])
def test_conv_halo(shape, splits, tile, np_, dgrad):
    """Halo-staged 3x3 fprop / data gradient (tiles 16-23) against fp64: partial blocks, blocks
    across image boundaries, bands of rows, partial column tiles (128- and 64-column tiles),
    32- and 64-channel chunks and split-K."""
    C = _C()
    N, H, W, Cin, K = shape
    cred, cout = (K, Cin) if dgrad else (Cin, K)
    if not _halo_ok("dgrad" if dgrad else "fprop", tile, W, cred, cout, np_):
        pytest.skip("shape outside this halo tile")
    g = torch.Generator().manual_seed(17)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64).requires_grad_(dgrad)
    w = torch.randn(K, Cin, 3, 3, generator=g, dtype=torch.float64) * 0.1
    y = F.conv2d(x, w, padding=1)
    w3 = _planes(w.float().permute(0, 2, 3, 1), np_)
    tol = 1e-5 if np_ in (2, 3) else 2e-2
    if not dgrad:
        out = torch.empty(N, H, W, K, device="cuda")
        slab = torch.empty(splits * N * H * W * K, device="cuda") if splits > 1 else None
        x3 = _planes(x.float().permute(0, 2, 3, 1), np_)
        C.conv_x3_fprop(x3, w3, out, slab, 1, 1, splits, tile, True, False, **_osc(x3, w3))
        torch.cuda.synchronize()
        assert rel_err(out.permute(0, 3, 1, 2), y.detach()) < tol
    else:
        dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
        (gx,) = torch.autograd.grad(y, x, dy)
        dx = torch.empty(N, H, W, Cin, device="cuda")
        slab = torch.empty(splits * N * H * W * Cin, device="cuda") if splits > 1 else None
        dz3 = _planes(dy.float().permute(0, 2, 3, 1), np_)
        C.conv_x3_dgrad(dz3, w3, dx, slab, 1, 1, splits, tile, True, False, **_osc(dz3, w3))
        torch.cuda.synchronize()
        assert rel_err(dx.permute(0, 3, 1, 2), gx) < tol


@pytest.mark.parametrize("shape", HALO_SHAPES + [(4, 32, 32, 8, 64)])
@pytest.mark.parametrize("splits", [1, 5])
@pytest.mark.parametrize("tile", [16, 17])
@pytest.mark.parametrize("np_", [3, 2, 1])
def test_conv_halo_wgrad(shape, splits, tile, np_):
    """Halo-staged 3x3 weight gradient (tiles 16/17: 64/32-pixel chunks) against fp64."""
    C = _C()
    N, H, W, Cin, K = shape
    if not _halo_ok("wgrad", tile, W, Cin, K):
        pytest.skip("shape outside this halo tile")
    g = torch.Generator().manual_seed(18)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64)
    w = (torch.randn(K, Cin, 3, 3, generator=g, dtype=torch.float64) * 0.1).requires_grad_(True)
    y = F.conv2d(x, w, padding=1)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (gw,) = torch.autograd.grad(y, w, dy)
    dw = torch.empty(K, 3, 3, Cin, device="cuda")
    slab = torch.empty(splits * K * 9 * Cin, device="cuda") if splits > 1 else None
    x3, dz3 = _planes(x.float().permute(0, 2, 3, 1), np_), _planes(dy.float().permute(0, 2, 3, 1), np_)
    C.conv_x3_wgrad(x3, dz3, dw, slab, 1, 1, splits, tile, False, **_osc(x3, dz3))
    torch.cuda.synchronize()
    assert rel_err(dw.permute(0, 3, 1, 2), gw) < (1e-5 if np_ in (2, 3) else 2e-2)


def test_halo_rejects_unsupported_shapes():
    """A halo tile on a conv it cannot run fails loudly (no silent substitute)."""
    C = _C()
    x3 = torch.zeros(1, 1, 8, 8, 24, device="cuda", dtype=torch.bfloat16)   # 24 channels: not a 16-multiple
    w3 = torch.zeros(1, 16, 3, 3, 24, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(1, 8, 8, 16, device="cuda")
    with pytest.raises(RuntimeError):
        C.conv_x3_fprop(x3, w3, out, None, 1, 1, 1, 16, True, False)


@pytest.mark.parametrize("shape", [(4, 8, 8, 64, 128, 1, 1, 0), (2, 8, 8, 64, 64, 1, 2, 0), (4, 16, 16, 32, 64, 3, 1, 1)])
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("tile", [5, 6, 16])
@pytest.mark.parametrize("obf", [False, True])
def test_conv_x3_dgrad_with_addend(shape, splits, tile, obf):
    """dx = dgrad + add, folded into the epilogue (one split) or the split-K reduction (GradJoin's
    residual-gradient sum); fp32 output with 3 planes, bf16 output with 1 plane."""
    C = _C()
    N, H, W, Cin, K, R, st, pd = shape
    if tile == 16 and (R != 3 or st != 1):
        pytest.skip("halo tiles are 3x3/s1 only")
    np_ = 1 if obf else 3
    g = torch.Generator().manual_seed(17 + splits)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64).requires_grad_(True)
    w = torch.randn(K, Cin, R, R, generator=g, dtype=torch.float64) * 0.1
    y = F.conv2d(x, w, stride=st, padding=pd)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (gx,) = torch.autograd.grad(y, x, dy)
    add = torch.randn(N, H, W, Cin, generator=g)
    dt = torch.bfloat16 if obf else torch.float32
    addd = add.to(dt).cuda()
    dx = torch.empty(N, H, W, Cin, device="cuda", dtype=dt)
    slab = torch.empty(splits * N * H * W * Cin, device="cuda") if splits > 1 else None
    C.conv_x3_dgrad(_planes(dy.float().permute(0, 2, 3, 1), np_), _planes(w.float().permute(0, 2, 3, 1), np_), dx,
                    slab, st, pd, splits, tile, True, False, addd)
    torch.cuda.synchronize()
    ref = gx.permute(0, 2, 3, 1) + addd.double().cpu()
    assert rel_err(dx, ref) < (2e-2 if obf else 1e-5)


# ----------------------------------------------------------------- position-major small-image kernels
POS_SHAPES = [
    # N, H, W, C, K   (3x3, stride 1, pad 1)
    (40, 2, 2, 64, 96),      # partial image group (40 of 64) and a partial column tile
    (70, 4, 4, 64, 128),     # 4x4: position blocks of 4 / 8, partial group
    (8, 2, 4, 32, 32),       # non-square image
    (256, 2, 2, 512, 512),   # VGG-11 layers 6-7 at batch 256
    (64, 4, 4, 256, 512),    # VGG-11 layer 4 (a quarter of the batch)
]


def _pos_ok(kind, tile, h, w, cred, cout):
    from distributed_pytorch_amd.engine import pos_ok

    return pos_ok(kind, tile, h, w, cred, cout)


@pytest.mark.parametrize("shape", POS_SHAPES)
@pytest.mark.parametrize("splits", [1, 4])
@pytest.mark.parametrize("tile", [24, 25, 26, 27, 28, 29])
@pytest.mark.parametrize("np_", [3, 2, 1])
@pytest.mark.parametrize("dgrad", [False, True])
def test_conv_pos(shape, splits, tile, np_, dgrad):
    """Position-major 3x3 fprop / data gradient with padding taps skipped (tiles 24-29) against
    fp64, and bit-for-bit against the halo kernel with the same channel chunk and split count (a
    skipped tap only adds exact zeros there)."""
    C = _C()
    N, H, W, Cin, K = shape
    cred, cout = (K, Cin) if dgrad else (Cin, K)
    kind = "dgrad" if dgrad else "fprop"
    if not _pos_ok(kind, tile, H, W, cred, cout):
        pytest.skip("shape outside this tile")
    g = torch.Generator().manual_seed(19)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64).requires_grad_(dgrad)
    w = torch.randn(K, Cin, 3, 3, generator=g, dtype=torch.float64) * 0.1
    y = F.conv2d(x, w, padding=1)
    w3 = _planes(w.float().permute(0, 2, 3, 1), np_)
    tol = 1e-5 if np_ in (2, 3) else 2e-2
    halo = 18 if tile == 29 else 19  # the halo tile with the same channel chunk (16 / 32)
    outs = []
    for t in (tile, halo):
        if not dgrad:
            out = torch.empty(N, H, W, K, device="cuda")
            slab = torch.empty(splits * N * H * W * K, device="cuda") if splits > 1 else None
            x3 = _planes(x.float().permute(0, 2, 3, 1), np_)
            C.conv_x3_fprop(x3, w3, out, slab, 1, 1, splits, t, True, False, **_osc(x3, w3))
        else:
            dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(20), dtype=torch.float64)
            out = torch.empty(N, H, W, Cin, device="cuda")
            slab = torch.empty(splits * N * H * W * Cin, device="cuda") if splits > 1 else None
            dz3 = _planes(dy.float().permute(0, 2, 3, 1), np_)
            C.conv_x3_dgrad(dz3, w3, out, slab, 1, 1, splits, t, True, False, **_osc(dz3, w3))
        torch.cuda.synchronize()
        outs.append(out)
    if not dgrad:
        ref = y.detach()
    else:
        (ref,) = torch.autograd.grad(y, x, dy)
    assert rel_err(outs[0].permute(0, 3, 1, 2), ref) < tol
    if _halo_ok(kind, halo, W, cred, cout):
        assert torch.equal(outs[0], outs[1])


def test_pos_rejects_unsupported_shapes():
    """A position-major tile on an image with too many staged pixels fails loudly."""
    C = _C()
    x3 = torch.zeros(1, 32, 8, 8, 32, device="cuda", dtype=torch.bfloat16)  # 8x8: more than 12 staged pixels
    w3 = torch.zeros(1, 32, 3, 3, 32, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(32, 8, 8, 32, device="cuda")
    with pytest.raises(RuntimeError):
        C.conv_x3_fprop(x3, w3, out, None, 1, 1, 1, 25, True, False)


# ----------------------------------------------------------------- BN statistics from the conv epilogue
EPI_SHAPES = [
    # N, H, W, C, K, R, stride, pad
    (3, 9, 9, 32, 48, 3, 1, 1),      # partial row tile, partial column tile
    (2, 14, 14, 64, 128, 1, 1, 0),   # 1x1 (ResNet bottleneck)
    (4, 8, 8, 16, 64, 3, 2, 1),      # strided
    (3, 9, 9, 64, 48, 3, 1, 1),      # 64-channel chunks (halo tiles 22/23)
]


@pytest.mark.parametrize("shape", EPI_SHAPES)
@pytest.mark.parametrize("tile", [0, 1, 5, 7, 11, 14, 16, 17, 18, 19, 20, 21, 22, 23])
@pytest.mark.parametrize("np_", [1, 2, 3])
@pytest.mark.parametrize("posmajor", [0, 1])
def test_conv_epilogue_bn_stats(shape, tile, np_, posmajor):
    """A one-split forward conv writes per-(row tile, channel) (mean, M2) of its output; the BN
    finalize from them gives the batch statistics of the output -- against fp64 statistics of the
    stored output (for bf16 output the statistics are those of the fp32 accumulators: within bf16
    rounding of the stored values' statistics)."""
    C_ = _C()
    N, H, W, Cin, K, R, st, pd = shape
    if tile >= 16 and (R != 3 or st != 1 or not _halo_ok("fprop", tile, W, Cin, K, np_)):
        pytest.skip("halo tiles are 3x3/s1 only")
    if tile >= 16 and posmajor:
        pytest.skip("halo tiles ignore the row order")
    g = torch.Generator().manual_seed(23)
    x = torch.randn(N, H, W, Cin, generator=g)
    w = torch.randn(K, R, R, Cin, generator=g) * 0.1 + 0.02  # nonzero channel means
    P = (H + 2 * pd - R) // st + 1
    out = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16 if np_ == 1 else torch.float32)
    rows = C_.conv_stats_rows(tile)
    nblk = (N * P * P + rows - 1) // rows
    stats = torch.full((2 * nblk * K,), float("nan"), device="cuda")
    x3, w3 = _planes(x, np_), _planes(w, np_)
    C_.conv_x3_fprop(x3, w3, out, None, st, pd, 1, tile, True, posmajor, stats, **_osc(x3, w3))
    dev = dict(device="cuda", dtype=torch.float32)
    gamma, beta = torch.rand(K, **dev) + 0.5, torch.randn(K, **dev)
    rm, rv, nbt = torch.zeros(K, **dev), torch.ones(K, **dev), torch.zeros(1, dtype=torch.int64, device="cuda")
    mean, invstd, scale, shift = (torch.empty(K, **dev) for _ in range(4))
    C_.bn_finalize(stats, nblk, rows, N * P * P, gamma, beta, None, rm, rv, nbt, mean, invstd, scale, shift, 0.1, 1e-5)
    torch.cuda.synchronize()
    zz = out.double().cpu().reshape(-1, K)
    mu, var = zz.mean(0), zz.var(0, unbiased=False)
    tol = 1e-5 if np_ in (2, 3) else 2e-3
    assert rel_err(mean, mu) < tol
    assert rel_err(invstd, torch.rsqrt(var + 1e-5)) < 10 * tol
    assert rel_err(rv, 0.9 + 0.1 * zz.var(0, unbiased=True)) < 10 * tol
    assert int(nbt.item()) == 1


def test_conv_epilogue_stats_refused_with_split_k():
    C_ = _C()
    x3 = torch.zeros(1, 2, 8, 8, 64, device="cuda", dtype=torch.bfloat16)
    w3 = torch.zeros(1, 64, 3, 3, 64, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(2, 8, 8, 64, device="cuda", dtype=torch.bfloat16)
    slab = torch.empty(4 * out.numel(), device="cuda")
    with pytest.raises(RuntimeError):
        C_.conv_x3_fprop(x3, w3, out, slab, 1, 1, 4, 0, True, 0, torch.empty(2 * 64 * 64, device="cuda"))


@pytest.mark.parametrize("shape", [(8, 56, 56, 64, 256), (4, 14, 14, 1024, 256), (2, 7, 7, 2048, 512),
                                   (3, 9, 11, 40, 72), (1, 3, 3, 512, 2048)])
@pytest.mark.parametrize("stats", [False, True])
def test_stream_tile_1x1_fprop(shape, stats):
    """The persistent streaming GEMM (tile 30, 1x1/s1 bf16 forward): bitwise the output (and BN
    statistics partials) of the implicit-GEMM tile 7 with the same 256x128 tile and k order, and
    against fp64 on the bf16-rounded operands."""
    C = _C()
    N, H, W, Cin, K = shape
    g = torch.Generator().manual_seed(41)
    x = torch.randn(N, H, W, Cin, generator=g).bfloat16()
    w = (torch.randn(K, 1, 1, Cin, generator=g) * 0.1).bfloat16()
    M = N * H * W
    outs = {}
    for tile in (7, 30):
        out = torch.full((N, H, W, K), float("nan"), device="cuda", dtype=torch.bfloat16)
        st = torch.zeros(2 * (-(-M // 256)) * K, device="cuda") if stats else None
        C.conv_x3_fprop(x.cuda().unsqueeze(0), w.cuda().unsqueeze(0), out, None, 1, 0, 1, tile, True, False, st)
        torch.cuda.synchronize()
        outs[tile] = (out.cpu(), st.cpu() if st is not None else None)
    assert torch.equal(outs[7][0], outs[30][0])
    if stats:
        assert torch.equal(outs[7][1], outs[30][1])
    ref = (x.double().reshape(M, Cin) @ w.double().reshape(K, Cin).t()).reshape(N, H, W, K)
    assert rel_err(outs[30][0].float(), ref) < 1e-2


@pytest.mark.parametrize("shape", [(8, 56, 56, 256, 64), (4, 14, 14, 256, 1024), (2, 7, 7, 512, 2048),
                                   (3, 9, 11, 72, 40)])
@pytest.mark.parametrize("add", [False, True])
def test_stream_tile_1x1_dgrad(shape, add):
    """Tile 30 as the data gradient of a 1x1/s1 conv (W read row-contiguous, transposed LDS reads):
    bitwise the implicit-GEMM tile 7 DGRAD, against fp64, and with a folded second contribution."""
    C = _C()
    N, H, W, Cin, K = shape  # forward conv Cin -> K; the data gradient maps dZ [.., K] to dX [.., Cin]
    g = torch.Generator().manual_seed(43)
    dz = torch.randn(N, H, W, K, generator=g).bfloat16()
    w = (torch.randn(K, 1, 1, Cin, generator=g) * 0.1).bfloat16()
    extra = torch.randn(N, H, W, Cin, generator=g).bfloat16()
    outs = {}
    for tile in (7, 30):
        dx = torch.full((N, H, W, Cin), float("nan"), device="cuda", dtype=torch.bfloat16)
        C.conv_x3_dgrad(dz.cuda().unsqueeze(0), w.cuda().unsqueeze(0), dx, None, 1, 0, 1, tile, True, False,
                        extra.cuda() if add else None)
        torch.cuda.synchronize()
        outs[tile] = dx.cpu()
    assert torch.equal(outs[7], outs[30])
    ref = (dz.double().reshape(-1, K) @ w.double().reshape(K, Cin)).reshape(N, H, W, Cin)
    if add:
        ref = ref + extra.double()
    assert rel_err(outs[30].float(), ref) < 1e-2
