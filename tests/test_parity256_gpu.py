"""The benchmark's exact kernel configurations, checked against fp64 autograd.

bench.py trains VGG-11 at batch 256 with the measured per-layer conv configurations of
tuning/mi355x.json (halo tiles, split-K counts up to 512, ...).  Smaller-batch parity tests run the
heuristic configurations instead, so here ONE full training step at batch 256 — forward, softmax-CE,
backward, fused SGD — is compared tensor by tensor with ``VGG11().double()`` autograd + torch SGD on
the same weights and data (reference: main.py:32-36, model.py:11-46):

* every conv call of the step (8 fprop, 7 dgrad, 8 wgrad) at its tuned configuration, fed with
  random operands, vs fp64 conv: rel ≤ 1e-5 (a wrong tile, split or reduction shows up as O(1));
* the loss, all 34 parameter gradients and the 34 parameter updates of the whole step.  A
  random-init VGG-11 with BN at batch 256 is ill-conditioned (stock torch fp32 on CPU is off from
  fp64 by up to ~3e-2 on single gradient tensors, measured): a perturbation at fp32 rounding level
  flips some 2x2 max-pool / ReLU decisions and moves single gradient tensors by 1e-3..1e-2.  The
  yardstick is that floor, measured per tensor (torch fp32, and fp64 and torch fp32 runs on inputs
  and weights perturbed by 2^-24):
  x3, h2 (fp16 pairs) and the fp32 MFMA path must stay within 4x of it on every tensor, and on
  the median tensor be no worse than torch fp32;
* the layer-0 weight gradient, whose reduction runs over all 256·32·32 = 262,144 output pixels
  (the longest sum in the step), at the tuned x3 config vs fp32 MFMA vs fp64.
"""
import json
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

N = 256


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _reference(sd=None, data_seed=256):
    """fp64 autograd + torch SGD, one step from state_dict ``sd`` (default: seed-1 init)."""
    from distributed_pytorch_amd.models import VGG11

    torch.manual_seed(1)
    m = VGG11().double()
    if sd is not None:
        m.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in sd.items()})
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(data_seed)
    x = torch.randn(N, 3, 32, 32, generator=g, dtype=torch.float64)
    t = torch.randint(0, 10, (N,), generator=g)
    loss = F.cross_entropy(m(x), t)
    loss.backward()
    grads = {n: p.grad.clone() for n, p in m.named_parameters()}
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    opt.step()
    new = {n: p.detach().clone() for n, p in m.named_parameters()}
    return dict(sd0=sd0, x=x, t=t, loss=float(loss), grads=grads, new=new)


@pytest.fixture(scope="module")
def reference():
    return _reference()


def _perturbed_errors(ref, seed, dtype):
    """The step's own conditioning: autograd (fp64, or stock torch fp32 on the CPU) on inputs and
    weights perturbed by random relative noise of 2^-24 (one fp32 rounding), vs the unperturbed
    fp64 step.  A random-init VGG-11 with BN amplifies such noise by orders of magnitude on some
    tensors (a 2x2 max-pool or ReLU decision flips under it), so a per-tensor error is only
    meaningful against this floor; the fp32 samples also carry fp32 rounding in every layer, as
    any fp32 implementation does."""
    from distributed_pytorch_amd.models import VGG11

    g = torch.Generator().manual_seed(seed)
    pert = lambda t: (t * (1 + 2.0 ** -24 * (2 * torch.rand(t.shape, generator=g, dtype=torch.float64) - 1))).to(dtype)
    m = VGG11().to(dtype)
    m.load_state_dict({k: pert(v) if v.is_floating_point() else v for k, v in ref["sd0"].items()})
    F.cross_entropy(m(pert(ref["x"])), ref["t"]).backward()
    return {n: (_rel(p.grad, ref["grads"][n]) if ref["grads"][n].abs().max() >= 1e-7 else None)
            for n, p in m.named_parameters()}


def _torch_fp32_errors(ref):
    from distributed_pytorch_amd.models import VGG11

    m = VGG11()
    m.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in ref["sd0"].items()})
    F.cross_entropy(m(ref["x"].float()), ref["t"]).backward()
    zero = {n: p.grad.abs().max().item() for n, p in m.named_parameters() if ref["grads"][n].abs().max() < 1e-7}
    return {n: (_rel(p.grad, ref["grads"][n]) if ref["grads"][n].abs().max() >= 1e-7 else None)
            for n, p in m.named_parameters()}, zero


def _engine_step(ref, impl):
    from distributed_pytorch_amd.engine import VGGEngine, conv_key, tuning_table

    e = VGGEngine("VGG11", "cuda", max_batch=N, impl=impl)
    # the tuned table must cover every conv call of the step at this batch (no heuristic fallback)
    tab = tuning_table()
    for i, l in enumerate(e.spec.convs):
        for kind in ("fprop", "dgrad", "wgrad"):
            if kind == "dgrad" and i == 0:
                continue
            impl_i = e._layer_impl(i)
            k = conv_key(impl_i, kind, N, l.hw, l.cin_pad, l.cout)
            if impl_i == "h2" and k not in tab:  # the fp16-pair kernels run x3's measured plan
                k = conv_key("x3", kind, N, l.hw, l.cin_pad, l.cout)
            assert k in tab, f"no tuned entry for {k}"
    e.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in ref["sd0"].items()})
    old = {n: e._to_torch_layout(n, e.params[n]).cpu().double() for n in ref["grads"]}
    x4 = torch.zeros(N, 32, 32, 4)
    x4[..., :3] = ref["x"].float().permute(0, 2, 3, 1)
    loss = float(e.forward_backward(x4.cuda(), ref["t"].cuda()).item())
    grads = {n: e._to_torch_layout(n, e.grads[n]).cpu() for n in ref["grads"]}
    e.sgd_step()
    e.finish_step()
    torch.cuda.synchronize()
    new = {n: e._to_torch_layout(n, e.params[n]).cpu().double() for n in ref["grads"]}
    return loss, grads, old, new


def _errors(reference, impls=("fp32", "x3", "h2"), dump="gpurun_out/parity256_errors.json"):
    out = {}
    for impl in impls:
        loss, grads, old, new = _engine_step(reference, impl)
        ge, ue, zero = {}, {}, {}
        for n, gref in reference["grads"].items():
            if gref.abs().max() < 1e-7:  # conv biases: analytically zero gradient (BN follows)
                ge[n] = None
                zero[n] = grads[n].abs().max().item()
            else:
                ge[n] = _rel(grads[n], gref)
            # update error, absolute, and what fp32 arithmetic allows for it: the gradient's error
            # times lr, plus one rounding of the parameter itself (p - lr*buf is formed in fp32)
            dref = reference["new"][n] - reference["sd0"][n]
            err = ((new[n] - old[n]) - dref).abs().max().item()
            gabs = 0.0 if ge[n] is None else ge[n] * gref.abs().max().item()
            allow = 0.1 * max(gabs, 1e-6) + 2.0 ** -23 * reference["new"][n].abs().max().item()
            ue[n] = [err, allow]
        out[impl] = dict(loss=abs(loss - reference["loss"]) / abs(reference["loss"]), grads=ge, updates=ue, zero=zero)
    tg, tz = _torch_fp32_errors(reference)
    out["torch_fp32"] = dict(grads=tg, zero=tz)
    out["perturbed"] = ([dict(dtype="fp64", grads=_perturbed_errors(reference, sd, torch.float64)) for sd in (1, 2)]
                        + [dict(dtype="fp32", grads=_perturbed_errors(reference, sd, torch.float32)) for sd in (3, 4)])
    # per tensor: the largest error any reference-grade computation of this step shows
    out["floor"] = {n: (None if e is None else max([e] + [p["grads"][n] for p in out["perturbed"]]))
                    for n, e in out["torch_fp32"]["grads"].items()}
    os.makedirs("gpurun_out", exist_ok=True)
    with open(dump, "w") as f:
        json.dump(out, f, indent=1)
    return out


@pytest.fixture(scope="module")
def errors(reference):
    return _errors(reference)


def _check_grade(errors, impl):
    floor, tref = errors["floor"], errors["torch_fp32"]["grads"]
    ratios = []
    for n, e in errors[impl]["grads"].items():
        if e is None:
            continue
        assert e <= 4.0 * floor[n] + 1e-5, (n, e, floor[n])
        ratios.append(e / max(tref[n], 1e-12))
    ratios.sort()
    assert ratios[len(ratios) // 2] <= 1.5, ratios


@pytest.mark.parametrize("impl", ["fp32", "x3", "h2"])
def test_loss_matches_fp64(errors, impl):
    assert errors[impl]["loss"] < 1e-5, errors[impl]["loss"]


@pytest.mark.parametrize("impl", ["fp32", "x3", "h2"])
def test_all_gradients_fp32_grade(errors, impl):
    """Every gradient tensor within 4x of the step's error floor (the largest error among torch
    fp32 and fp64 / fp32 runs perturbed at fp32 rounding level), and the median tensor no worse
    than torch fp32 itself."""
    _check_grade(errors, impl)


def _trained_state(steps=200):
    """The reference-layout state after ``steps`` training steps (lr 0.1, momentum 0.9, wd 1e-4,
    batch 256) on the bench's synthetic data: weights and BN statistics far from the random init,
    where activations, gradient magnitudes and the fp16-pair bounds are those of real training.
    Trained with stock torch on the GPU (deterministic MIOpen algorithms), so the state -- and every
    error measured from it -- does not move when the framework's own kernels change."""
    from distributed_pytorch_amd.data import synthetic_cifar
    from distributed_pytorch_amd.models import VGG11

    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    torch.manual_seed(1)
    m = VGG11().cuda()
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    train = synthetic_cifar(N * 50, 0)
    imgs = train.images.cuda().permute(0, 3, 1, 2).float().div_(255.0).sub_(0.5).div_(0.25)
    labels = train.labels.cuda()
    for i in range(steps):
        j = (i % 50) * N
        opt.zero_grad(set_to_none=True)
        F.cross_entropy(m(imgs[j:j + N]), labels[j:j + N]).backward()
        opt.step()
    torch.cuda.synchronize()
    return {k: v.detach().cpu() for k, v in m.state_dict().items()}


@pytest.fixture(scope="module")
def trained_errors():
    ref = _reference(_trained_state(), data_seed=512)
    return _errors(ref, impls=("fp32", "x3", "h2"), dump="gpurun_out/parity256_trained_errors.json")


@pytest.mark.parametrize("impl", ["x3", "h2"])
def test_parity_at_trained_state(trained_errors, impl):
    """the same whole-step fp64 comparison from a TRAINED state (200 steps of
    training on the bench's synthetic data, _trained_state), where the fixed fp16-pair scales and
    the data-gradient bounds meet the magnitudes of real training rather than of the random init.

    The yardstick is the engine's own exact-fp32 path (fp32 MFMA convs, same BatchNorm kernels) at
    the same state: at a trained state every engine path, that one included, sits ~2.5-3x further
    from fp64 than stock torch CPU fp32 on the median tensor -- a property of the folded BatchNorm
    apply y = z*scale + shift (its rounding scales with |mean * scale| once |mean| > sigma; torch's
    CPU kernel differs; tools/fwd_precision.py, docs/PERF_NOTES.md round 6), not of the conv
    arithmetic.  x3 / h2 must be fp32-grade against that path: loss to 1e-5, every tensor within 4x
    of max(step floor, exact-fp32 engine error), the median tensor within 1.5x of the exact-fp32
    engine's error, updates to fp32 rounding."""
    e = trained_errors
    assert e[impl]["loss"] < 1e-5, e[impl]["loss"]
    ratios = []
    for n, err in e[impl]["grads"].items():
        if err is None:
            continue
        base = max(e["floor"][n], e["fp32"]["grads"][n])
        assert err <= 4.0 * base + 1e-5, (n, err, base)
        ratios.append(err / max(e["fp32"]["grads"][n], 1e-12))
    ratios.sort()
    assert ratios[len(ratios) // 2] <= 1.5, ratios
    for n, (err, allow) in e[impl]["updates"].items():
        assert err <= 2.0 * allow, (n, err, allow)


def test_exact_fp32_engine_at_trained_state(trained_errors):
    """The engine's exact-fp32 path against stock torch fp32 at the trained state: tracked, with a
    loose bound (the BatchNorm-apply gap in test_parity_at_trained_state's docstring is ~2.5-3x on
    the median tensor; a regression well beyond it fails)."""
    e = trained_errors
    tref = e["torch_fp32"]["grads"]
    r = sorted(err / max(tref[n], 1e-12) for n, err in e["fp32"]["grads"].items() if err is not None)
    assert e["fp32"]["loss"] < 1e-5 and r[len(r) // 2] <= 5.0, r


@pytest.mark.parametrize("impl", ["fp32", "x3", "h2"])
def test_zero_gradients_at_rounding_level(errors, impl):
    """Conv biases ahead of BN have an analytically zero gradient; what is left is the cancellation
    of the BN backward sums, which any fp32 computation shows: within 4x of torch fp32's own
    residue (or 1e-5)."""
    tz = errors["torch_fp32"]["zero"]
    for n, v in errors[impl]["zero"].items():
        assert v <= max(1e-5, 4.0 * tz[n]), (n, v, tz[n])


@pytest.mark.parametrize("impl", ["fp32", "x3", "h2"])
def test_all_updates_match_fp64(errors, impl):
    # an update is -lr * (g + wd * p) on the first step (conv biases: g analytically 0)
    for n, (err, allow) in errors[impl]["updates"].items():
        assert err <= 2.0 * allow, (n, err, allow)


CALLS = [(i, k) for i in range(8) for k in ("fprop", "dgrad", "wgrad") if not (i == 0 and k == "dgrad")]


_ENGINES = {}


def _bench_engine(impl):
    from distributed_pytorch_amd.engine import VGGEngine

    if impl not in _ENGINES:
        e = VGGEngine("VGG11", "cuda", max_batch=N, impl=impl)
        e.init_parameters(seed=1)
        _ENGINES[impl] = e
    return _ENGINES[impl]


@pytest.mark.parametrize("impl", ["x3", "fp32", "h2"])
@pytest.mark.parametrize("layer,kind", CALLS)
def test_conv_call_at_bench_config(impl, layer, kind):
    """One conv call of the step exactly as the engine issues it (tuned tile/splits, its own
    workspaces and operand buffers) on random operands vs fp64.  Both the x3 planes path and the
    exact-fp32 MFMA path: each call's error is at fp32 rounding level (<= 1e-5 of the output's
    scale), so the per-tensor spread of whole-step gradient errors (test_all_gradients_fp32_grade)
    comes from the step's conditioning, not from any one reduction."""
    from distributed_pytorch_amd import _ext

    C = _ext.require()
    e = _bench_engine(impl)
    l = e.spec.convs[layer]
    g = torch.Generator().manual_seed(100 * layer + len(kind))
    cin = l.cin
    act = torch.randn(N, l.hw, l.hw, cin, generator=g)
    w = e._to_torch_layout(f"{l.conv_key}.weight", e.params[f"{l.conv_key}.weight"]).cpu().double()  # OIHW
    x4 = None
    if layer == 0:
        x4 = torch.zeros(N, 32, 32, 4)
        x4[..., :3] = act
        x4 = x4.cuda()
        if e.x0p is not None:
            C.pad_split8(x4, e.x0p)
    elif e.planes[layer]:
        C.split_planes(act.cuda().contiguous().view(-1), e.a3[layer - 1].view(e.np, -1),
                       e.h2_sa if e.np == 2 else 1.0)
    else:
        e.a[layer - 1].copy_(act.cuda())
    xd = act.permute(0, 3, 1, 2).double()
    torch.cuda.synchronize()
    if kind == "fprop":
        e._conv_fwd(layer, x4, N, reduce=True)
        out = e.z[layer].cpu().permute(0, 3, 1, 2).double()
        ref = F.conv2d(xd, w, padding=1)
    else:
        dz = torch.randn(N, l.hw, l.hw, l.cout, generator=g)
        if e.planes[layer] and e.np == 2:
            # fp16 pairs: the scale follows the bound word BN backward would have written
            import math

            B = float(dz.abs().max())
            e.dzb[layer] = torch.tensor([B], dtype=torch.float32).view(torch.int32).item()
            C.split_planes(dz.cuda().view(-1), e.dz3[layer].view(2, -1), 2.0 ** (14 - math.frexp(B)[1]))
        elif e.planes[layer]:
            C.split_planes(dz.cuda().view(-1), e.dz3[layer].view(3, -1))
        else:
            e.dz[layer].copy_(dz.cuda())
        dzd = dz.permute(0, 3, 1, 2).double()
        if kind == "dgrad":
            s = e._conv_dgrad(layer, N)
            shp = e.g[layer - 1].shape
            if s > 1:
                out = e.slab[: s * e.g[layer - 1].numel()].view(s, *shp).double().sum(0).cpu()
            else:
                out = e.g[layer - 1].cpu().double()
            out = out.permute(0, 3, 1, 2)
            ref = torch.nn.grad.conv2d_input(xd.shape, w, dzd, padding=1)
        else:
            e._conv_wgrad(layer, x4, N)
            out = e._to_torch_layout(f"{l.conv_key}.weight", e.grads[f"{l.conv_key}.weight"]).cpu().double()
            ref = torch.nn.grad.conv2d_weight(xd, w.shape, dzd, padding=1)
    torch.cuda.synchronize()
    err = _rel(out, ref)
    assert err < 1e-5, (layer, kind, e.conv_config(layer, kind, N), err)


def test_layer0_wgrad_full_reduction_accuracy():
    """wgrad of layer 0 at the bench's tuned x3 config (262,144-long reduction) vs fp32 MFMA vs fp64."""
    from distributed_pytorch_amd import _ext
    from distributed_pytorch_amd.engine import VGGEngine

    C = _ext.require()
    e = VGGEngine("VGG11", "cuda", max_batch=N, impl="x3")
    tile, splits, pm = e.conv_config(0, "wgrad", N)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(N, 3, 32, 32, generator=g)
    dz = torch.randn(N, 64, 32, 32, generator=g) * 1e-3
    ref = torch.nn.grad.conv2d_weight(x.double(), (64, 3, 3, 3), dz.double(), padding=1)  # [64,3,3,3]
    # x3 path: input padded to 8 channels and split into planes exactly as the engine does it
    x4 = torch.zeros(N, 32, 32, 4)
    x4[..., :3] = x.permute(0, 2, 3, 1)
    x4 = x4.cuda()
    xp = torch.zeros(3, N, 32, 32, 8, dtype=torch.bfloat16, device="cuda")
    C.pad_split8(x4, xp)
    dzd = dz.permute(0, 2, 3, 1).contiguous().cuda()
    dzp = torch.zeros(3, N, 32, 32, 64, dtype=torch.bfloat16, device="cuda")
    C.split_planes(dzd.view(-1), dzp.view(3, -1))
    dw3 = torch.zeros(64, 3, 3, 8, device="cuda")
    slab = torch.empty(max(1, splits) * dw3.numel(), device="cuda") if splits > 1 else None
    C.conv_x3_wgrad(xp, dzp, dw3, slab, 1, 1, splits, tile, pm)
    # exact fp32 MFMA path (4-channel padded input, as the fp32 engine runs layer 0)
    dw32 = torch.zeros(64, 3, 3, 4, device="cuda")
    s32 = 64
    slab32 = torch.empty(s32 * dw32.numel(), device="cuda")
    C.conv_wgrad(x4, dzd, dw32, slab32, 1, 1, s32, 0, False)
    torch.cuda.synchronize()
    r = ref.permute(0, 2, 3, 1)
    e3 = ((dw3[..., :3].double().cpu() - r).abs().max() / r.abs().max()).item()
    e32 = ((dw32[..., :3].double().cpu() - r).abs().max() / r.abs().max()).item()
    assert splits > 1  # the tuned plan really splits the reduction
    assert e3 < 1e-5, e3
    assert e3 <= 4.0 * e32 + 1e-7, (e3, e32)
