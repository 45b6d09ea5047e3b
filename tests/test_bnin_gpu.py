"""Consumer-side BatchNorm, forward (conv_x3.hip BNIN): the forward 3x3 conv
applies the previous layer's BN + ReLU (+ 2x2 max-pool) while staging its operand from that layer's
fp32 z.  It must be bit for bit the bn_apply pass followed by the plane conv: the conv output, the
epilogue statistics and the operand planes it stores for the weight-gradient conv.  Oracle of the
layer chain itself: /root/reference/model.py:16,18-25.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from distributed_pytorch_amd import _ext

    return _ext.require()


def _planes(t, np_):
    C = _C()
    out = torch.empty(np_, *t.shape, device="cuda", dtype=torch.bfloat16)
    C.split_planes(t.contiguous().cuda(), out)
    return out


# (N, Hz, Wz, C, K, pool): the VGG-11 forward calls at batch 256 and odd small ones (partial tiles,
# halo rows across images)
SHAPES = [(256, 32, 32, 64, 128, True), (256, 16, 16, 128, 256, True), (256, 8, 8, 256, 256, False),
          (256, 8, 8, 256, 512, True), (256, 4, 4, 512, 512, False), (3, 16, 16, 64, 96, True),
          (5, 6, 6, 32, 64, False), (2, 12, 12, 96, 40, True)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("splits", [1, 2])
@pytest.mark.parametrize("tile", [17, 19])
@pytest.mark.parametrize("np_", [3, 1])
def test_bn_on_load_matches_apply_then_conv(shape, splits, tile, np_):
    C = _C()
    N, Hz, Wz, Cin, K, pool = shape
    H, W = (Hz // 2, Wz // 2) if pool else (Hz, Wz)
    g = torch.Generator().manual_seed(23)
    z = (torch.randn(N, Hz, Wz, Cin, generator=g) * 2 + 0.3).cuda()
    scale = (torch.randn(Cin, generator=g) * 0.7).cuda()  # both signs (the pooled max/min path)
    shift = torch.randn(Cin, generator=g).cuda()
    w3 = _planes(torch.randn(K, 3, 3, Cin, generator=g) * 0.05, np_)
    # reference: bn_apply -> planes, then the plane conv
    a3 = torch.empty(np_, N, H, W, Cin, device="cuda", dtype=torch.bfloat16)
    C.bn_apply(z, a3, scale, shift, pool)
    ref = torch.empty(N, H, W, K, device="cuda")
    rows = C.conv_stats_rows(tile)
    nst = 2 * ((N * H * W + rows - 1) // rows) * K
    st_ref = torch.zeros(nst, device="cuda") if splits == 1 else None
    slab = torch.zeros(splits * N * H * W * K, device="cuda") if splits > 1 else None
    C.conv_x3_fprop(a3, w3, ref, slab, 1, 1, splits, tile, True, 0, st_ref)
    # BN on load
    a3w = torch.zeros_like(a3)
    out = torch.empty_like(ref)
    st = torch.zeros(nst, device="cuda") if splits == 1 else None
    slab2 = torch.zeros_like(slab) if slab is not None else None
    C.conv_x3_fprop_bnin(z, pool, scale, shift, a3w, w3, out, slab2, splits, tile, st)
    torch.cuda.synchronize()
    if splits > 1:
        assert torch.equal(slab2, slab)  # (slabs are left unreduced)
    assert torch.equal(a3w, a3), "operand planes differ from bn_apply's"
    if splits == 1:
        assert torch.equal(out, ref)
        assert torch.equal(st, st_ref)


def test_bn_on_load_refuses_other_tiles():
    C = _C()
    z = torch.zeros(2, 8, 8, 64, device="cuda")
    sc = torch.ones(64, device="cuda")
    w3 = torch.zeros(3, 64, 3, 3, 64, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(2, 4, 4, 64, device="cuda")
    with pytest.raises(RuntimeError):
        C.conv_x3_fprop_bnin(z, True, sc, sc, None, w3, out, None, 1, 16)


# (N, H, W, K, C, pool): the VGG-11 data-gradient calls at batch 256 (layers 1-4) and odd small ones
BWD_SHAPES = [(256, 16, 16, 128, 64, True), (256, 8, 8, 256, 128, False), (256, 8, 8, 256, 256, True),
              (256, 4, 4, 512, 256, False), (3, 8, 8, 64, 96, True), (5, 6, 6, 32, 64, False)]


@pytest.mark.parametrize("shape", BWD_SHAPES)
@pytest.mark.parametrize("splits", [1, 2])
@pytest.mark.parametrize("tile", [17, 19, 20, 21])
def test_bn_bwd_on_load_matches_apply_then_dgrad(shape, splits, tile):
    """dgrad with the BN backward applied on load (conv_x3.hip BNIN 3/4) is bitwise bn_bwd's apply
    pass followed by the plane dgrad: dx (or its slabs) and the dz planes it stores."""
    from distributed_pytorch_amd.engine import halo_ok

    C = _C()
    N, H, W, K, Cin, pool = shape
    if not halo_ok("dgrad", tile, W, K, Cin):
        pytest.skip("shape outside this halo tile")
    g = torch.Generator().manual_seed(29)
    z = (torch.randn(N, H, W, K, generator=g) * 2 + 0.3).cuda()
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    gout = torch.randn(N, Ho, Wo, K, generator=g).cuda()
    scale = (torch.randn(K, generator=g) * 0.7).cuda()
    shift = torch.randn(K, generator=g).cuda()
    mean, invstd = torch.randn(K, generator=g).cuda(), (torch.rand(K, generator=g) + 0.5).cuda()
    gamma = torch.randn(K, generator=g).cuda()
    w3 = _planes(torch.randn(K, 3, 3, Cin, generator=g) * 0.05, 3)
    part = torch.zeros(C.bn_part_floats(N * Ho * Wo, K, True), device="cuda")
    coef = torch.empty(3 * K, device="cuda")
    dg, db, dbias = (torch.empty(K, device="cuda") for _ in range(3))
    # reference: three-kernel BN backward writing dz planes, then the plane dgrad
    dz3 = torch.empty(3, N, H, W, K, device="cuda", dtype=torch.bfloat16)
    gg = gout.clone()
    C.bn_bwd(gg, 1, gg, z, scale, shift, mean, invstd, gamma, part, coef, dg, db, dbias, dz3, pool)
    ref = torch.empty(N, H, W, Cin, device="cuda")
    slab = torch.zeros(splits * N * H * W * Cin, device="cuda") if splits > 1 else None
    C.conv_x3_dgrad(dz3, w3, ref, slab, 1, 1, splits, tile, False, 0)
    # on load (the coefficients of the statistics-only pass must equal the reference's)
    coef2 = torch.empty_like(coef)
    gg2 = gout.clone()
    C.bn_bwd_stats(gg2, 1, gg2, z, scale, shift, mean, invstd, gamma, part, coef2, dg, db, dbias, pool)
    dz3w = torch.zeros_like(dz3)
    out = torch.empty_like(ref)
    slab2 = torch.zeros_like(slab) if slab is not None else None
    C.conv_x3_dgrad_bnin(gg2, z, pool, scale, shift, coef2, dz3w, w3, out, slab2, splits, tile)
    torch.cuda.synchronize()
    assert torch.equal(coef2, coef)
    assert torch.equal(dz3w, dz3), "dz planes differ from bn_bwd_apply's"
    if splits > 1:
        assert torch.equal(slab2, slab)
    else:
        assert torch.equal(out, ref)


@pytest.mark.parametrize("impl", ["x3", "bf16"])
@pytest.mark.parametrize("bwd", ["1", "0"])
def test_engine_step_bitwise_with_and_without_bn_on_load(monkeypatch, impl, bwd):
    """Two VGG-11 training steps (batch 256: the tuned halo tiles) with the BN applied on load
    (forward, and backward when bwd) are bitwise the steps with the apply passes: loss, gradients,
    parameters, BN statistics."""
    from distributed_pytorch_amd.engine import VGGEngine

    torch.manual_seed(0)
    x = torch.zeros(256, 32, 32, 4, device="cuda")
    x[..., :3] = torch.randn(256, 32, 32, 3, device="cuda")
    t = torch.randint(0, 10, (256,), device="cuda")
    res = []
    for on in ("1", "0"):
        monkeypatch.setenv("DPA_BN_ON_LOAD", on)
        monkeypatch.setenv("DPA_BN_BWD_ON_LOAD", bwd if on == "1" else "0")
        eng = VGGEngine("VGG11", "cuda", max_batch=256, impl=impl)
        eng.init_parameters(seed=1)
        used = [eng._bnin(i, 256) for i in range(8)]
        assert any(used) == (on == "1"), used
        used_b = [eng._bnin_bwd(i, 256) for i in range(8)]
        assert any(used_b) == (on == "1" and bwd == "1" and impl == "x3"), used_b
        for _ in range(2):
            eng.forward_backward(x, t)
            eng.sgd_step()
            eng.finish_step()
        torch.cuda.synchronize()
        eng.check_signals()
        res.append((eng.loss.clone(), eng.grads.flat.clone(), eng.params.flat.clone(), eng.buffers.flat.clone()))
    for a, b in zip(*res):
        assert torch.equal(a, b)
