"""Plain-PyTorch reference implementation of the native kernel API (same names, same signatures,
same in-place output semantics as ``distributed_pytorch_amd._C``).

Used (a) as the CPU backend of the training engine, so the whole distributed harness — sync
modes, buckets, checkpointing — runs and is tested on CPU with gloo, and (b) as the numerics
oracle the HIP kernels are checked against.  Tensors follow the native layouts: NHWC
activations, KRSC conv weights.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

CHUNK = 64


def _nchw(t):
    return t.permute(0, 3, 1, 2)


def _nhwc(t):
    return t.permute(0, 2, 3, 1)


# ---------------------------------------------------------------- optimizer / elementwise
def sgd_flat(p, g, buf, lr, momentum, wd, gscale, first, offset=0, count=-1, planes=None):
    if count < 0:
        count = p.numel() - offset
    sl = slice(offset, offset + count)
    pp, gg, bb = p[sl], g[sl], buf[sl]
    d = gg * gscale + wd * pp
    if first:
        bb.copy_(d)
    else:
        bb.mul_(momentum).add_(d)
    pp.sub_(lr * bb)
    if planes is not None:
        planes[:, sl].copy_(split_bf16(pp, planes.shape[0]))


def split_bf16(x, np_):
    """fp32 -> [np_, *x.shape] bf16 planes (round-to-nearest-even), the HIP split's semantics."""
    out, r = [], x.float()
    for _ in range(np_):
        h = r.to(torch.bfloat16)
        out.append(h)
        r = r - h.float()
    return torch.stack(out)


def mean_of_w(inp, out, W):
    out.copy_(inp.view(W, -1).mean(0))


# ---------------------------------------------------------------- convolution
def conv_splits(Kred, splits):
    return max(1, min(max(1, splits), -(-Kred // 32)))


def conv_fprop(x, w, out, slab, stride, pad, splits=1, tile=0, dgrad=False, reduce=True, posmajor=False):
    if dgrad:  # w: the original conv's weights [C_in_of_this_gemm=K_orig, R, S, C_orig]
        w = w.flip(1, 2).permute(3, 1, 2, 0)
    y = _nhwc(F.conv2d(_nchw(x), _nchw(w), stride=stride, padding=pad))
    eff = conv_splits(w.shape[1] * w.shape[2] * w.shape[3], splits)
    if eff > 1 and not reduce:  # mirror the native contract: the slabs sum to the result
        n = y.numel()
        slab[:eff * n].zero_()
        slab[:n].copy_(y.reshape(-1))
        return
    out.copy_(y)


def conv_wgrad(x, dz, dw, slab, stride, pad, splits=1, tile=0, posmajor=False):
    K, R, S, C = dw.shape
    gw = torch.nn.grad.conv2d_weight(_nchw(x), (K, C, R, S), _nchw(dz), stride=stride, padding=pad)
    dw.copy_(_nhwc(gw))


def wflip(w, wd):
    wd.copy_(w.flip(1, 2).permute(3, 1, 2, 0))


# ---------------------------------------------------------------- batch norm
def bn_part_floats(M, C, bwd):
    return (3 if bwd else 2) * C * ((M + CHUNK - 1) // CHUNK)


def bn_fwd_stats(src, nsplit, z, part, gamma, beta, bias, rmean, rvar, nbt, mean, invstd, scale, shift, momentum,
                 eps):
    C = z.shape[-1]
    if nsplit > 1:
        z.copy_(src[:nsplit * z.numel()].view(nsplit, -1).sum(0).view(z.shape))
    zz = z.reshape(-1, C).double()
    n = zz.shape[0]
    mu = zz.mean(0)
    var = zz.var(0, unbiased=False)
    iv = torch.rsqrt(var + eps)
    mean.copy_(mu)
    invstd.copy_(iv)
    scale.copy_(gamma.double() * iv)
    shift.copy_(beta.double() - mu * gamma.double() * iv)
    if rmean is not None:
        b = bias.double() if bias is not None else 0.0
        unb = var * n / max(n - 1, 1)
        rmean.copy_((1 - momentum) * rmean.double() + momentum * (mu + b))
        rvar.copy_((1 - momentum) * rvar.double() + momentum * unb)
    if nbt is not None:
        nbt.add_(1)


def bn_eval_params(gamma, beta, bias, rmean, rvar, scale, shift, eps):
    s = gamma * torch.rsqrt(rvar + eps)
    scale.copy_(s)
    b = bias if bias is not None else 0.0
    shift.copy_(beta + (b - rmean) * s)


def _act(u, act, res):
    if act == 1:
        return u
    if act == 2:
        u = u + res.reshape(u.shape)
    return torch.relu(u)


def bn_apply(z, a, scale, shift, pool, act=0, res=None, mask=None):  # mask: native only (CPU keeps res)
    y = _act(z * scale + shift, act, res)
    if pool:
        y = _nhwc(F.max_pool2d(_nchw(y), 2, 2))
    a.copy_(y.reshape(a.shape))


def bn_bwd(gsrc, nsplit, g, z, scale, shift, mean, invstd, gamma, part, coef, dgamma, dbeta, dbias, dz, pool,
           act=0, res=None, dres=None, sig=None, sig_val=0, g2=None, mask=None):
    N, H, W, C = z.shape
    if nsplit > 1:
        g.copy_(gsrc[:nsplit * g.numel()].view(nsplit, -1).sum(0).view(g.shape))
    else:
        g = gsrc
    if g2 is not None:  # a second contribution to the same gradient (native: summed on load)
        g = g + g2
    with torch.enable_grad():
        u = (z * scale + shift).detach().requires_grad_(True)  # BN output, pre-activation
        y = _act(u, act, res)
        if pool:
            y = _nhwc(F.max_pool2d(_nchw(y), 2, 2))
        (dy,) = torch.autograd.grad(y, u, g.reshape(y.shape))
    if act == 2:
        dres.copy_(dy.reshape(dres.shape))
    xh = (z - mean) * invstd
    M = N * H * W
    sdy = dy.reshape(-1, C).sum(0)
    sdx = (dy * xh).reshape(-1, C).sum(0)
    sx = xh.reshape(-1, C).sum(0)
    k1 = gamma * invstd
    out = k1 * (dy - sdy / M - xh * sdx / M)
    dz.copy_(out)
    dgamma.copy_(sdx)
    dbeta.copy_(sdy)
    if dbias is not None:
        dbias.copy_(-k1 * sx * sdx / M)


def wgrad0_part_floats(N):
    return 1


def bn_bwd_wgrad0(gsrc, nsplit, g, z, scale, shift, mean, invstd, gamma, part, coef, dgamma, dbeta, dbias, x, wpart,
                  dw):
    """Layer-0 backward (native: bn.hip bn_bwd_wgrad0_kernel): BN backward with ReLU + 2x2 max-pool
    routing, then the 3x3/s1/p1 weight gradient on the input x [N,H,W,4] (channels >= 3 zero)."""
    dz = torch.empty_like(z)
    bn_bwd(gsrc, nsplit, g, z, scale, shift, mean, invstd, gamma, part, coef, dgamma, dbeta, dbias, dz, True)
    cin = 3
    w = torch.nn.grad.conv2d_weight(_nchw(x[..., :cin]), (z.shape[-1], cin, 3, 3), _nchw(dz), padding=1)
    dw.zero_()
    dw[..., :cin].copy_(w.permute(0, 2, 3, 1))


# ---------------------------------------------------------------- classifier head
def fc_ce_train(x, w, b, target, loss_row, dlogits, dx, dw, db, loss_out, loss_accum, bn_z=None, bn_scale=None,
                bn_shift=None):
    B = x.shape[0]
    if bn_z is not None:  # features from the last conv's z: BN + ReLU + 2x2 max-pool, written to x
        x.copy_(torch.relu(bn_z * bn_scale + bn_shift).reshape(B, 4, -1).amax(1))
    logits = x @ w.t() + b
    lse = torch.logsumexp(logits, 1)
    lr = lse - logits.gather(1, target.view(-1, 1)).squeeze(1)
    loss_row.copy_(lr)
    p = torch.softmax(logits, 1)
    p[torch.arange(B), target] -= 1.0
    p /= B
    dlogits.copy_(p.reshape(dlogits.shape))
    dx.copy_(p @ w)
    dw.copy_(p.t() @ x)
    db.copy_(p.sum(0))
    l = lr.mean()
    loss_out.reshape(-1)[0] = l
    if loss_accum is not None:
        loss_accum.reshape(-1)[0] += l


def fc_ce_eval(x, w, b, target, loss_row, correct_row, logits=None, acc=None):
    lg = x @ w.t() + b
    lse = torch.logsumexp(lg, 1)
    lr = lse - lg.gather(1, target.view(-1, 1)).squeeze(1)
    loss_row.copy_(lr)
    correct_row.copy_((lg.argmax(1) == target).to(correct_row.dtype))
    if logits is not None:
        logits.copy_(lg)
    if acc is not None:
        acc[0] += lr.mean()
        acc[1] += correct_row.sum().to(acc.dtype)


# ---------------------------------------------------------------- data
_M1 = 0x9E3779B97F4A7C15
_M2 = 0xBF58476D1CE4E5B9
_M3 = 0x94D049BB133111EB
_MASK = (1 << 64) - 1


def _mix64(z):
    z = (z + _M1) & _MASK
    z = ((z ^ (z >> 30)) * _M2) & _MASK
    z = ((z ^ (z >> 27)) * _M3) & _MASK
    return z ^ (z >> 31)


def aug_params(seed, salt, b, pad):
    """(dy, dx, flip) of sample slot b — bit-identical to the HIP kernel's hash."""
    h = _mix64((seed & _MASK) ^ _mix64((salt * 0x100000001B3 + b) & _MASK))
    span = 2 * pad + 1
    return h % span, (h >> 16) % span, (h >> 40) & 1


def augment(images, idx, labels, out, target, pad, train, seed, salt, mean, std):
    B = idx.numel()
    Hs, Ws = images.shape[1], images.shape[2]
    m = torch.tensor(mean, dtype=torch.float32)
    inv = 1.0 / torch.tensor(std, dtype=torch.float32)
    src = images[idx.long()].float() * (1.0 / 255.0)  # B H W 3
    res = torch.zeros(B, Hs, Ws, 4)
    for b in range(B):
        if train:
            dy, dx, flip = aug_params(seed, salt, b, pad)
        else:
            dy, dx, flip = pad, pad, 0
        padded = torch.zeros(Hs + 2 * pad, Ws + 2 * pad, 3)
        padded[pad:pad + Hs, pad:pad + Ws] = src[b]
        crop = padded[dy:dy + Hs, dx:dx + Ws]
        if flip:
            crop = crop.flip(1)
        res[b, :, :, :3] = (crop - m) * inv
    out.copy_(res.reshape(out.shape))
    if target is not None:
        target.copy_(labels[idx.long()])
