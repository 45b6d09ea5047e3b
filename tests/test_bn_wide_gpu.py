"""bf16 BatchNorm apply passes with 16-byte lanes (csrc/kernels/bn_wide.hip) vs bn.hip's 8-byte-lane
kernels they replace: forward BN+ReLU / BN / BN+residual+ReLU (with the ReLU mask) and the backward
apply (ReLU recomputed from z, identity, second gradient summed on load, the add+ReLU dy pass),
all BITWISE equal, on shapes that take the capped-grid path (grid stride a multiple of C/8), the
uncapped path, and a C % 8 != 0 fallback.  The backward reduce with 16-byte lanes partitions rows
differently from bn.hip's (same per-element math, other summation order): its statistics agree to
fp32 rounding and the dy it stores (the residual gradient) is bitwise equal."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(2, 7, 7, 2048), (4, 14, 14, 64), (128, 28, 28, 64), (16, 28, 28, 1000), (2, 5, 5, 12)]
# tensors large enough for the 1024-thread reduce geometry (M * C / 4 > 3M), incl. C/8 not dividing 1024
RED_SHAPES = [(128, 56, 56, 64), (64, 14, 14, 1024), (128, 7, 7, 2048), (16, 28, 28, 1000)]


def _ext():
    from distributed_pytorch_amd import _ext as E

    return E.require()


def _inputs(shape, seed):
    g = torch.Generator().manual_seed(seed)
    N, H, W, C = shape
    b = lambda: (torch.randn(N, H, W, C, generator=g) * 2).to(torch.bfloat16).cuda()
    f = lambda s=1.0, o=0.0: (torch.randn(C, generator=g) * s + o).cuda()
    return dict(z=b(), res=b(), gz=b(), g2=b(), scale=f(0.5, 1.0), shift=f(), mean=f(), invstd=f(0.1, 1.0).abs(),
                gamma=f(0.3, 1.0))


def _run(monkeypatch, wide, fn):
    monkeypatch.setenv("DPA_BN_WIDE", "1" if wide else "0")
    out = fn()
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("shape", SHAPES)
def test_bn_apply_wide_bitwise(monkeypatch, shape, act):
    K = _ext()
    d = _inputs(shape, 1 + act)

    def fwd():
        a = torch.empty_like(d["z"])
        mask = torch.zeros(d["z"].numel() // 4, dtype=torch.uint8, device="cuda") if act == 2 else None
        K.bn_apply(d["z"], a, d["scale"], d["shift"], False, act, d["res"] if act == 2 else None, mask=mask)
        return a, mask

    a0, m0 = _run(monkeypatch, False, fwd)
    a1, m1 = _run(monkeypatch, True, fwd)
    assert torch.equal(a0.view(torch.int16), a1.view(torch.int16))
    if act == 2:
        assert torch.equal(m0, m1)


@pytest.mark.parametrize("act,with_g2,use_mask", [(0, False, False), (0, True, False), (1, False, False),
                                                  (1, True, False), (2, False, True), (2, False, False)])
@pytest.mark.parametrize("shape", SHAPES)
def test_bn_bwd_apply_wide_bitwise(monkeypatch, shape, act, with_g2, use_mask):
    monkeypatch.setenv("DPA_BN_WIDE_RED", "0")  # the reduce of both runs is bn.hip's (bitwise comparison)
    _bwd_compare(monkeypatch, shape, act, with_g2, use_mask, exact=True)


@pytest.mark.parametrize("act,with_g2,use_mask", [(0, False, False), (0, True, False), (1, True, False),
                                                  (2, False, True), (2, True, True), (2, False, False)])
@pytest.mark.parametrize("shape", RED_SHAPES)
def test_bn_bwd_reduce_wide(monkeypatch, shape, act, with_g2, use_mask):
    _bwd_compare(monkeypatch, shape, act, with_g2, use_mask, exact=False)


def _bwd_compare(monkeypatch, shape, act, with_g2, use_mask, exact):
    K = _ext()
    d = _inputs(shape, 10 + act)
    N, H, W, C = shape
    mask = None
    if use_mask:
        mask = torch.zeros(d["z"].numel() // 4, dtype=torch.uint8, device="cuda")
        K.bn_apply(d["z"], torch.empty_like(d["z"]), d["scale"], d["shift"], False, 2, d["res"], mask=mask)

    def bwd():
        dz = torch.empty_like(d["z"])
        dres = torch.empty_like(d["z"]) if act == 2 else None
        part = torch.zeros(K.bn_part_floats(N * H * W, C, True), device="cuda")
        coef = torch.empty(4 * C, device="cuda")
        dgamma, dbeta = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
        K.bn_bwd(d["gz"], 1, d["gz"], d["z"], d["scale"], d["shift"], d["mean"], d["invstd"], d["gamma"], part, coef,
                 dgamma, dbeta, None, dz, False, act, d["res"] if act == 2 and mask is None else None, dres,
                 g2=d["g2"] if with_g2 else None, mask=mask)
        return dz, dres, coef, dgamma, dbeta

    r0 = _run(monkeypatch, False, bwd)
    r1 = _run(monkeypatch, True, bwd)
    names = ["dz", "dres", "coef", "dgamma", "dbeta"]
    for name, x, y in zip(names, r0, r1):
        if x is None:
            assert y is None
            continue
        if exact or name == "dres":
            assert torch.equal(x.view(torch.int16) if x.dtype == torch.bfloat16 else x,
                               y.view(torch.int16) if y.dtype == torch.bfloat16 else y), name
        elif name == "dz":  # coefficients differ in the last fp32 bits: a bf16 ulp (or cancellation noise)
            xf, yf = x.float(), y.float()
            assert ((xf - yf).abs() <= xf.abs() * 2 ** -7 + xf.abs().max() * 1e-5).all(), name
        else:
            rel = ((x - y).abs().max() / x.abs().max().clamp_min(1e-30)).item()
            assert rel < 1e-4, (name, rel)

