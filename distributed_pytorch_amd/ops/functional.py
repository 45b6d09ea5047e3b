"""Autograd functions over the gfx950 kernels, for generic ``nn.Module`` models (ResNet-50 etc.).

The VGG engine (engine.py) drives the kernels through a static, hand-scheduled step; this module
exposes the same kernels to PyTorch autograd so arbitrary NHWC conv/BN networks can be built from
them ("autograd.Functions over the kernels, used for generic nn.Module paths").

Layout and precision contract (all tensors NHWC, contiguous):
  conv2d_nhwc   x [N,H,W,C] (C % 8 == 0), w fp32 [K,R,S,C] (master weights) -> z [N,P,Q,K].
                impl "bf16": activations, conv outputs and their gradients are bf16 tensors that
                the MFMA kernels read/write directly (one bf16 plane; fp32 accumulation; the
                weight is rounded to bf16 per call); fp32 inputs are rounded on entry.
                impl "x3": fp32 activations, split into three bf16 planes inside the op
                (fp32-grade results, see conv_x3.hip).  No conv bias (every conv feeds a BN).
  bn_act_nhwc   z (bf16 or fp32) -> act(BN(z) [+ residual]) in z's dtype; statistics and affine in
                fp32; act 0 = ReLU, 1 = none, 2 = ReLU(. + res).  Training mode updates running
                stats in place (momentum, unbiased var) and num_batches_tracked; backward
                recomputes the activation mask from z (+res).
On CPU the same functions run the fp32 CPU oracle (ops/cpu_ref.py) so models are testable here;
on a GPU the native extension is required (loud failure, no silent fallback).
"""
from __future__ import annotations

import json
import math
import os
from typing import Callable, Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from .. import _ext
from . import cpu_ref

ACT = {"relu": 0, "none": 1, "add_relu": 2}
NPLANES = {"bf16": 1, "x3": 3}


def _native(t: torch.Tensor) -> bool:
    return t.is_cuda


class _Workspace:
    """Per-device scratch reused by consecutive ops (all on the compute stream, so stream order
    makes reuse safe): split-K slabs and the BN reduction workspace (zero-initialised once)."""

    def __init__(self):
        self.bufs: Dict[Tuple[str, torch.device], torch.Tensor] = {}

    def get(self, kind: str, numel: int, device, zero: bool = False) -> torch.Tensor:
        key = (kind, torch.device(device))
        t = self.bufs.get(key)
        if t is None or t.numel() < numel:
            t = (torch.zeros if zero else torch.empty)(max(numel, 64), device=device, dtype=torch.float32)
            self.bufs[key] = t
        return t


WS = _Workspace()


def split_planes(x: torch.Tensor, np_: int) -> torch.Tensor:
    """[NP, *x.shape] bf16 operand planes of x (a bf16 x with NP == 1 is used as is)."""
    if x.dtype == torch.bfloat16:
        if np_ != 1:
            raise ValueError("a bf16 tensor only provides one operand plane")
        return x.contiguous().unsqueeze(0)
    out = torch.empty((np_,) + tuple(x.shape), device=x.device, dtype=torch.bfloat16)
    _ext.require().split_planes(x.contiguous().float(), out)
    return out


def weight_planes(w: torch.Tensor, np_: int) -> torch.Tensor:
    """Operand planes of a conv weight: the cached copy the optimizer keeps current
    (``w._dpa_planes``, refreshed inside the fused SGD kernel, see parallel/ddp.py) when it is
    still valid for this tensor version, else a fresh split."""
    pl = getattr(w, "_dpa_planes", None)
    if pl is not None and pl.shape[0] == np_ and getattr(w, "_dpa_planes_ver", -1) == w._version:
        return pl
    return split_planes(w, np_)


def grad_slot(p: torch.Tensor) -> Optional[torch.Tensor]:
    """Where a parameter gradient may be written directly: the optimizer arena view
    (``p._dpa_grad_slot()``), when the parameter has no gradient yet this step and was used exactly
    once in this forward (``p._dpa_uses`` holds the forward's TOTAL use count by the time backward
    runs).  The view is handed back to autograd, whose AccumulateGrad adopts it as ``p.grad``
    instead of running a copy / add kernel per parameter.  A parameter used more than once gets a
    fresh tensor per use; autograd sums them and the DDP hook moves the sum into the arena."""
    slot = getattr(p, "_dpa_grad_slot", None)
    if slot is None or p.grad is not None or getattr(p, "_dpa_uses", 0) != 1:
        return None
    return slot()


def note_use(p: torch.Tensor) -> int:
    """Count uses of a parameter in the current forward (the DDP wrapper resets the count)."""
    n = getattr(p, "_dpa_uses", 0) + 1
    p._dpa_uses = n
    return n


# ------------------------------------------------------------------ conv launch configuration
# Per-call (tile, splits, posmajor): measured table (tuning/generic_mi355x.json, written by the
# autotuner: ``set_autotune(True)``, e.g. ``bench_resnet.py --autotune``), else a heuristic.
TABLE_PATH = os.environ.get("DPA_GENERIC_TABLE") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "generic_mi355x.json")  # env: A/B
_table: Optional[Dict[str, list]] = None
_chosen: Dict[str, Tuple[int, int, bool]] = {}
_AUTOTUNE = {"on": os.environ.get("DPA_AUTOTUNE", "0") == "1", "dirty": False}
N_TILES = 16


def set_autotune(on: bool):
    _AUTOTUNE["on"] = bool(on)


def _table_get() -> Dict[str, list]:
    global _table
    if _table is None:
        _table = {}
        if os.environ.get("DPA_NO_TUNING", "0") != "1" and os.path.exists(TABLE_PATH):
            with open(TABLE_PATH) as f:
                _table = json.load(f)
    return _table


def save_tuning_table(path: Optional[str] = None):
    """Merge the autotuned entries into the JSON table (atomic replace)."""
    path = path or TABLE_PATH
    cur = {}
    if os.path.exists(path):
        with open(path) as f:
            cur = json.load(f)
    cur.update(_table_get())
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(dict(sorted(cur.items())), f, indent=0)
    os.replace(tmp, path)
    _AUTOTUNE["dirty"] = False


def halo_candidates(kind: str, geom: tuple, np_: int = 1) -> Tuple[int, ...]:
    """Halo-staged tiles (conv_x3.hip, ids >= 16) that can run this conv call: 3x3, stride 1,
    pad 1 only, channel / row-width / plane-count limits as in engine.halo_ok."""
    from ..engine import HALO_TILES, HALO_WGRAD_TILES, halo_ok

    N, H, W, C, K, R, S, stride, pad = geom
    if (R, S, stride, pad) != (3, 3, 1, 1):
        return ()
    if kind == "wgrad":
        return tuple(t for t in HALO_WGRAD_TILES if halo_ok("wgrad", t, W, C, K))
    cred, cout = (C, K) if kind == "fprop" else (K, C)
    return tuple(t for t in HALO_TILES if halo_ok(kind, t, W, cred, cout, np_))


STREAM_TILES = (30,)  # conv_x3.hip gemm_stream_kernel: 1x1 / stride 1 / pad 0 fprop + dgrad, bf16, one split


def stream_candidates(impl: str, kind: str, geom: tuple) -> Tuple[int, ...]:
    """The persistent streaming-GEMM tile when it can run this conv call."""
    N, H, W, C, K, R, S, stride, pad = geom
    ok = (impl == "bf16" and kind in ("fprop", "dgrad") and (R, S, stride, pad) == (1, 1, 1, 0) and C % 8 == 0
          and K % 8 == 0)
    return STREAM_TILES if ok else ()


def _autotune(key: str, kind: str, red: int, run: Callable[[int, int, bool], None],
              slab_bytes: Callable[[int], int], extra_tiles: Tuple[int, ...] = ()) -> Tuple[int, int, bool]:
    Kx = _ext.require()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    splits = (1, 2, 4, 8, 16, 32, 64, 128, 256) if kind == "wgrad" else (1, 2, 4, 8, 16)
    seen = set()
    for tile in tuple(range(N_TILES)) + tuple(extra_tiles):
        for s0 in splits:
            s = Kx.x3_splits(red, s0)
            for pm in (False, True):
                if (tile, s, pm) in seen or slab_bytes(s) > (512 << 20):
                    continue
                if tile in STREAM_TILES and (s > 1 or pm):  # one split, NHWC row order only
                    continue
                seen.add((tile, s, pm))
                try:
                    run(tile, s, pm)
                except RuntimeError:  # the tile refuses this call (shape / size limits): not a candidate
                    continue
                ev0.record()
                for _ in range(3):
                    run(tile, s, pm)
                ev1.record()
                ev1.synchronize()
                ms = ev0.elapsed_time(ev1) / 3
                if best is None or ms < best[3]:
                    best = [tile, s, pm, ms]
    _table_get()[key] = best
    _AUTOTUNE["dirty"] = True
    return best[0], best[1], best[2]


def choose_config(impl: str, kind: str, geom: tuple, M: int, Ngemm: int, Kred: int, hw_small: bool,
                  run: Optional[Callable[[int, int, bool], None]] = None,
                  slab_bytes: Optional[Callable[[int], int]] = None) -> Tuple[int, int, bool]:
    key = "|".join(str(v) for v in (impl, kind) + tuple(geom))
    c = _chosen.get(key)
    if c is not None:
        return c
    t = _table_get().get(key)
    if t is not None:
        c = (int(t[0]), int(t[1]), bool(t[2]))
    elif _AUTOTUNE["on"] and run is not None:
        c = _autotune(key, kind, M if kind == "wgrad" else Kred, run, slab_bytes,
                      halo_candidates(kind, geom, {"x3": 3, "h2": 2}.get(impl, 1)) + stream_candidates(impl, kind, geom))
    else:
        c = conv_config(kind, M, Ngemm, Kred, hw_small)
    _chosen[key] = c
    return c


_cfg_cache: Dict[tuple, Tuple[int, int, bool]] = {}


def conv_config(kind: str, M: int, Ngemm: int, Kred: int, hw_small: bool) -> Tuple[int, int, bool]:
    """(tile, splits, posmajor) heuristic for a GEMM view of a conv call: 128x128 single-stage
    tiles; split-K until ~2 blocks per CU; position-major rows for small spatial maps."""
    key = (kind, M, Ngemm, Kred, hw_small)
    c = _cfg_cache.get(key)
    if c is not None:
        return c
    cd = lambda a, b: (a + b - 1) // b
    if kind == "wgrad":
        tiles = cd(Ngemm, 128) * cd(Kred, 128)   # Kout x (R*S*C), reduction over M
        red = M
    else:
        tiles = cd(M, 128) * cd(Ngemm, 128)
        red = Kred
    s = 1
    while tiles * s < 512 and red // (2 * s) >= 256 and s < (512 if kind == "wgrad" else 16):
        s *= 2
    c = (5, s, hw_small)
    _cfg_cache[key] = c
    return c


# Deferred gradient contributions (GradJoin with ``defer``): data_ptr of a block input's gradient ->
# (that gradient, the addend).  The gradient's consumer -- the BN backward that produced the block
# input -- sums the addend on load (bn.hip ``g2``) instead of an elementwise add pass over it.
_DEFERRED: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}
DEFER_JOIN = True  # (tests switch it off: the add pass instead)
DEFER_STATS = {"summed_on_load": 0}  # BN backwards that consumed a deferred contribution (tests)
BN_RELU_MASK = True  # the add+ReLU forward stores a 1-bit ReLU mask the backward reads (tests: False)
# BN statistics from the producing conv's epilogue (conv_x3.hip epi_col_stats): a training conv with
# one split registers its (mean, M2) partials under its output's address; the BN that normalises
# that output finalizes from them instead of re-reading z (bn_stats_kernel).
EPI_STATS = True
# (entries hold the output tensor itself, so its address cannot be reused while the entry lives)
_STATS: Dict[int, Tuple[torch.Tensor, int, int, Tuple[int, int], torch.Tensor]] = {}
STATS_USED = {"epilogue": 0}  # BN forwards that finalized from conv epilogue partials (tests)


def clear_deferred():
    """Drop deferred contributions of an abandoned backward (called at every training forward)."""
    _DEFERRED.clear()
    _STATS.clear()


class GradJoin:
    """Joins the gradient contributions of several autograd nodes to ONE tensor without an
    elementwise add pass.  In a ResNet bottleneck the block input x feeds conv1 and the residual
    (the identity into bn3's add+ReLU, or the downsample conv): autograd would sum their gradients
    with an extra read-read-write pass over x's gradient.  Instead every contributor calls
    ``contribute``: all but the last stash their gradient and hand autograd None (a zero
    contribution, nothing to add); the last one folds the stash into its own output — inside the
    data-gradient split-K reduction when its conv splits K (``splitk_reduce_add``), else with one
    in-place add — and returns the sum.  Order-independent; ``reset()`` at every forward.

    ``defer`` (set per forward when the joined tensor was produced by a BN backward that can take a
    second gradient operand, ``bn_act_nhwc`` outputs): when the last contributor's data gradient
    has no split-K reduction to fold the stash into, the stash is not added at all but registered
    with the returned gradient; the producing BN backward sums it on load.  ``guard`` (a hook on
    the joined tensor) adds it explicitly if autograd summed the gradient with another one first."""

    __slots__ = ("n", "left", "buf", "defer", "key")

    def __init__(self, n: int):
        self.n = n
        self.defer = False
        self.key = None
        self.reset()

    def reset(self):
        self.left, self.buf = self.n, None

    def last(self) -> bool:
        return self.left == 1

    def stash(self, g: torch.Tensor) -> None:
        if self.buf is None:
            self.buf = g
        elif _native(g):
            _ext.require().add_inplace(self.buf, g.contiguous())
        else:
            self.buf = self.buf + g
        self.left -= 1

    def register(self, g: torch.Tensor, addend: torch.Tensor) -> None:
        """Defer ``addend`` to g's consumer (see class doc)."""
        self.key = g.data_ptr()
        _DEFERRED[self.key] = (g, addend)

    def guard(self, grad: torch.Tensor) -> Optional[torch.Tensor]:
        """Hook on the joined tensor: its total gradient is not the registered one (autograd summed
        other contributions into a new tensor) -> add the deferred addend here."""
        key, self.key = self.key, None
        if key is None or grad.data_ptr() == key:
            return None
        ent = _DEFERRED.pop(key, None)
        return grad if ent is None else grad + ent[1]

    def take(self) -> Optional[torch.Tensor]:
        """For the last contributor: the stashed sum (None if nothing was stashed); resets."""
        b = self.buf
        self.reset()
        return b

    def contribute(self, g: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """A contributor whose gradient is already materialised: stash it (returns None), or as the
        last one return it plus the stash."""
        if g is None:
            self.left -= 1
            return None if self.left > 0 else self.take()
        if not self.last():
            self.stash(g)
            return None
        b = self.take()
        if b is None:
            return g
        if _native(g):
            _ext.require().add_inplace(g, b.contiguous())
            return g
        return g + b


class Conv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride: int, pad: int, impl: str, join: Optional[GradJoin] = None,
                grad_mode: bool = True):
        N, H, W, Cx = x.shape
        K, R, S, C = w.shape  # C: the weight's (padded) input channels; x may carry fewer (network input)
        P, Q = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
        ctx.geom = (N, H, W, C, K, R, S, stride, pad, P, Q)
        ctx.impl = impl
        ctx.w_param = w
        ctx.cx = Cx
        ctx.join = join
        note_use(w)
        if not _native(x):
            if Cx != C:
                x = F.pad(x, (0, C - Cx))
            z = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), stride=stride, padding=pad)
            ctx.save_for_backward(x, w)
            return z.permute(0, 2, 3, 1).contiguous()
        Kx = _ext.require()
        np_ = NPLANES[impl]
        if Cx != C:
            # channel padding happens in the plane split (pad_split8): no padded fp32 copy of the input
            if C != 8 or Cx > 8:
                raise ValueError(f"conv2d_nhwc: input has {Cx} channels, weight {C} (only padding to 8 is fused)")
            xp = torch.empty(np_, N, H, W, 8, device=x.device, dtype=torch.bfloat16)
            Kx.pad_split8(x.float().contiguous(), xp)
        else:
            xp = split_planes(x, np_)
        wp = weight_planes(w, np_)
        act_dtype = torch.bfloat16 if np_ == 1 else torch.float32
        ctx.x_dtype = x.dtype if np_ == 3 else torch.bfloat16
        z = torch.empty(N, P, Q, K, device=x.device, dtype=act_dtype)
        geom = (N, H, W, C, K, R, S, stride, pad)

        def run(tile, s, pm, stats=None):
            slab = WS.get("slab", s * N * P * Q * K, x.device) if s > 1 else None
            Kx.conv_x3_fprop(xp, wp, z, slab, stride, pad, s, tile, True, pm, stats)

        cfg = choose_config(impl, "fprop", geom, N * P * Q, K, R * S * C, P * Q <= 16, run,
                            lambda s: 4 * s * N * P * Q * K)
        sk = Kx.x3_splits(R * S * C, cfg[1])
        # a training forward: grad mode as it was at the call site (it is off inside forward) and a
        # weight that needs a gradient.  An eval / no_grad forward registers nothing: its BN never
        # pops the entry, which would pin z until the next training step.
        rows = (Kx.conv_stats_rows(cfg[0]) if (EPI_STATS and sk == 1 and grad_mode and ctx.needs_input_grad[1])
                else 0)
        stats = None
        if rows > 0:
            nblk = (N * P * Q + rows - 1) // rows
            stats = torch.empty(2 * nblk * K, device=x.device, dtype=torch.float32)
            while len(_STATS) >= 64:  # a conv whose output no BN normalised (not in the supported models)
                _STATS.pop(next(iter(_STATS)))
            _STATS[z.data_ptr()] = (stats, nblk, rows, (N * P * Q, K), z)
        run(cfg[0], sk, cfg[2], stats)
        ctx.save_for_backward(xp, wp)
        return z

    @staticmethod
    def backward(ctx, dz):
        N, H, W, C, K, R, S, stride, pad, P, Q = ctx.geom
        geom = (N, H, W, C, K, R, S, stride, pad)
        a, b = ctx.saved_tensors
        dz = dz.contiguous()
        dx = dw = None
        if not _native(dz):
            x, w = a, b
            xn, wn = x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2)
            dzn = dz.permute(0, 3, 1, 2)
            if ctx.needs_input_grad[0]:
                dx = torch.nn.grad.conv2d_input(xn.shape, wn, dzn, stride=stride, padding=pad).permute(0, 2, 3, 1)
                if ctx.cx != C:
                    dx = dx[..., :ctx.cx]
            if ctx.needs_input_grad[1]:
                dw = torch.nn.grad.conv2d_weight(xn, wn.shape, dzn, stride=stride, padding=pad).permute(0, 2, 3, 1)
                slot = grad_slot(ctx.w_param)
                if slot is not None:
                    dw = slot.copy_(dw)
            if ctx.join is not None and ctx.needs_input_grad[0]:
                dx = ctx.join.contribute(dx.contiguous())
            return dx, dw, None, None, None, None, None
        Kx = _ext.require()
        xp, wp = a, b
        np_ = xp.shape[0]
        if np_ == 1 and dz.dtype != torch.bfloat16:
            dz = dz.to(torch.bfloat16)
        dzp = split_planes(dz, np_)
        join = ctx.join
        if ctx.needs_input_grad[0]:
            dx = torch.empty(N, H, W, C, device=dz.device, dtype=ctx.x_dtype)
            # last contributor of a GradJoin: the stashed gradient is folded into this data gradient
            addend = join.take() if (join is not None and join.last() and ctx.cx == C) else None

            def run_d(tile, s, pm, add=None):
                # add: dx = dgrad + stash, in the kernel's store (one split) or its split-K reduction
                slab = WS.get("slab", s * N * H * W * C, dz.device) if s > 1 else None
                Kx.conv_x3_dgrad(dzp, wp, dx, slab, stride, pad, s, tile, True, pm, add)

            cfg = choose_config(ctx.impl, "dgrad", geom, N * H * W, C, R * S * K, H * W <= 16, run_d,
                                lambda s: 4 * s * N * H * W * C)
            sk = Kx.x3_splits(R * S * K, cfg[1])
            if addend is not None:
                addend = addend.to(dx.dtype).contiguous()
            # no split-K reduction to fold the stash into: leave it to the producing BN backward
            defer = addend is not None and sk == 1 and join.defer
            run_d(cfg[0], sk, cfg[2], None if defer else addend)
            if defer:
                join.register(dx, addend)
        if ctx.needs_input_grad[1]:
            dw = grad_slot(ctx.w_param)
            if dw is None:
                dw = torch.empty(K, R, S, C, device=dz.device, dtype=torch.float32)

            def run_w(tile, s, pm):
                slab = WS.get("slab", s * K * R * S * C, dz.device) if s > 1 else None
                Kx.conv_x3_wgrad(xp, dzp, dw, slab, stride, pad, s, tile, pm)

            cfg = choose_config(ctx.impl, "wgrad", geom, N * P * Q, K, R * S * C, P * Q <= 16, run_w,
                                lambda s: 4 * s * K * R * S * C)
            run_w(cfg[0], Kx.x3_splits(N * P * Q, cfg[1]), cfg[2])
        if dx is not None and ctx.cx != C:
            dx = dx[..., :ctx.cx].contiguous()
        if join is not None and dx is not None and addend is None:
            dx = join.contribute(dx)  # not last (stash; autograd gets None), or a sliced input
        return dx, dw, None, None, None, None, None


def conv2d_nhwc(x: torch.Tensor, w: torch.Tensor, stride: int = 1, pad: int = 0, impl: str = "bf16",
                join: Optional[GradJoin] = None):
    """``join``: x's gradient is one of several contributions (GradJoin) to be summed without an
    extra pass."""
    if impl not in NPLANES:
        raise ValueError(f"impl must be one of {list(NPLANES)}")
    return Conv2dNHWC.apply(x.contiguous(), w, int(stride), int(pad), impl, join, torch.is_grad_enabled())


def _bn_coefs(K, z, gamma, beta, rmean, rvar, nbt, training: bool, momentum: float, eps: float):
    """(mean, invstd, scale, shift) of a BatchNorm over z [N,H,W,C]: from the producing conv's
    epilogue partials when it registered them, else a statistics pass (training), or the running
    statistics (eval).  Updates the running statistics in training."""
    N, H, W, C = z.shape
    dev = z.device
    # per-channel statistics in fp32 on GPU (bf16 activations too); the CPU oracle also runs fp64
    f32 = dict(device=dev, dtype=torch.float32 if _native(z) else z.dtype)
    mean, invstd, scale, shift = (torch.empty(C, **f32) for _ in range(4))
    st = _STATS.pop(z.data_ptr(), None) if training and _native(z) else None
    if st is not None and st[3] == (N * H * W, C):  # partials from the producing conv's epilogue
        K.bn_finalize(st[0], st[1], st[2], N * H * W, gamma, beta, None, rmean, rvar, nbt, mean, invstd, scale,
                      shift, momentum, eps)
        STATS_USED["epilogue"] += 1
    elif training:
        part = WS.get("bn_part", K.bn_part_floats(N * H * W, C, True), dev, zero=True) if _native(z) else None
        K.bn_fwd_stats(z, 1, z, part, gamma, beta, None, rmean, rvar, nbt, mean, invstd, scale, shift, momentum, eps)
    else:
        K.bn_eval_params(gamma, beta, None, rmean, rvar, scale, shift, eps)
    return mean, invstd, scale, shift


def _bn_grad_bufs(params, C: int, f32: dict):
    """dgamma / dbeta: the optimizer's direct slots when the parameters have them."""
    out = []
    for p in params:
        d = grad_slot(p)
        out.append(d if d is not None and d.dtype == f32["dtype"] else torch.empty(C, **f32))
    return out


class BnActNHWC(torch.autograd.Function):
    """Training / eval BatchNorm2d + activation on NHWC.  Optional fusions: ``pool`` (the output is
    max-pooled inside the pool's loads, ResNet stem) and ``rgamma``/``rbeta``/``rstate`` (act 2 only:
    ``res`` is the INPUT of a second BatchNorm -- the downsample branch -- whose BN is applied inside
    the add's loads; its backward runs here after this one's)."""

    @staticmethod
    def forward(ctx, z, gamma, beta, res, rmean, rvar, nbt, training: bool, momentum: float, eps: float, act: int,
                res_join: Optional[GradJoin] = None, pool: Optional[Tuple[int, int, int]] = None,
                rgamma=None, rbeta=None, rstate=None):
        N, H, W, C = z.shape
        dev = z.device
        K = _ext.require() if _native(z) else cpu_ref
        rbn = rgamma is not None
        if rbn:  # the residual branch's BN first (its statistics come from the downsample conv)
            rco = _bn_coefs(K, res, rgamma, rbeta, *rstate[:3], training, *rstate[3:])
        mean, invstd, scale, shift = _bn_coefs(K, z, gamma, beta, rmean, rvar, nbt, training, momentum, eps)
        arg = None
        mask = None
        if rbn:
            a = torch.empty_like(z)
            mask = torch.empty(z.numel() // 4, dtype=torch.uint8, device=dev)
            if not K.bn_apply_rbn(z, a, scale, shift, res, rco[2], rco[3], mask):
                r = torch.empty_like(res)
                K.bn_apply(res, r, rco[2], rco[3], False, 1)
                K.bn_apply(z, a, scale, shift, False, 2, r, mask=mask)
        elif pool is not None:
            # BN + ReLU applied inside the max-pool's loads (the ResNet stem): the BN output is never
            # stored; the pool's window positions route the backward
            k, st_, pd = pool
            a = torch.empty(N, conv_out(H, k, st_, pd), conv_out(W, k, st_, pd), C, device=dev, dtype=z.dtype)
            arg = torch.empty(a.shape, device=dev, dtype=torch.uint8)
            K.maxpool_fwd(z, a, arg, k, st_, pd, scale=scale, shift=shift)
        else:
            a = torch.empty_like(z)
            # add+ReLU in training on GPU: the kernel also writes the ReLU mask (1 byte per 4 channels),
            # which the backward reads instead of the residual
            mask = (torch.empty(z.numel() // 4, dtype=torch.uint8, device=dev)
                    if act == 2 and training and _native(z) and BN_RELU_MASK else None)
            K.bn_apply(z, a, scale, shift, False, act, res if act == 2 else None, mask=mask)
        ctx.act, ctx.training, ctx.pool, ctx.rbn = act, training, pool, rbn
        ctx.res_join = res_join
        ctx.params = (gamma, beta) + ((rgamma, rbeta) if rbn else ())
        if training:
            for p in ctx.params:
                note_use(p)
        rsave = (res, rgamma) + tuple(rco[:4]) if rbn else (None,) * 6
        ctx.save_for_backward(z, res if act == 2 and mask is None else None, mask, gamma, mean, invstd, scale, shift,
                              arg, *rsave)
        return a

    @staticmethod
    def backward(ctx, da):
        z, res, mask, gamma, mean, invstd, scale, shift, arg, rz, rgamma, rmean, rinvstd, rscale, rshift = \
            ctx.saved_tensors
        if not ctx.training:
            raise RuntimeError("bn_act_nhwc backward is only defined in training mode")
        # a deferred second contribution to da (GradJoin.register; never for the pooled form)
        ent = _DEFERRED.pop(da.data_ptr(), None) if ctx.pool is None else None
        da = da.contiguous()
        N, H, W, C = z.shape
        native = _native(z)
        K = _ext.require() if native else cpu_ref
        if ctx.pool is not None:  # the pool's gather first: the gradient of the (never stored) BN output
            k, st_, pd = ctx.pool
            dpre = torch.empty_like(z)
            K.maxpool_bwd(da, arg, dpre, k, st_, pd)
            da = dpre
        f32 = dict(device=z.device, dtype=torch.float32 if native else z.dtype)
        dz = torch.empty_like(z)
        dgamma, dbeta = _bn_grad_bufs(ctx.params[:2], C, f32)
        dres = torch.empty_like(z) if ctx.act == 2 else None
        part = WS.get("bn_part", K.bn_part_floats(N * H * W, C, True), z.device, zero=True) if native else None
        coef = torch.empty(4 * C, **f32)
        g2 = None  # ... summed on load by the kernels
        if ent is not None:
            if native and ent[1].dtype == da.dtype and ent[1].numel() == da.numel():
                g2 = ent[1]
                DEFER_STATS["summed_on_load"] += 1
            else:
                da = da + ent[1].view_as(da)
        K.bn_bwd(da, 1, da, z, scale, shift, mean, invstd, gamma, part, coef, dgamma, dbeta, None, dz, False, ctx.act,
                 res, dres, g2=g2, mask=mask)
        if ctx.rbn:  # dres is the gradient of the residual BN's output: its backward (identity act)
            drz = torch.empty_like(rz)
            drg, drb = _bn_grad_bufs(ctx.params[2:], C, f32)
            K.bn_bwd(dres, 1, dres, rz, rscale, rshift, rmean, rinvstd, rgamma, part, coef, drg, drb, None, drz, False,
                     1, None, None)
            return dz, dgamma, dbeta, drz, None, None, None, None, None, None, None, None, None, drg, drb, None
        if ctx.res_join is not None and dres is not None:
            dres = ctx.res_join.contribute(dres)
        return dz, dgamma, dbeta, dres, None, None, None, None, None, None, None, None, None, None, None, None


# BN + ReLU + max-pool as one forward pass (bn_act_nhwc ``pool``; tests: False = apply pass + pool)
FUSE_BN_POOL = True
# the downsample branch's BN applied inside the block's add + ReLU (bn_act_nhwc ``res_bn``; tests: False)
FUSE_RES_BN = True


def bn_act_nhwc(z, gamma, beta, running_mean, running_var, num_batches_tracked, training: bool = True,
                momentum: float = 0.1, eps: float = 1e-5, act: str = "relu", residual: Optional[torch.Tensor] = None,
                res_join: Optional[GradJoin] = None, pool: Optional[Tuple[int, int, int]] = None,
                res_bn=None):
    """``res_join``: the residual's gradient is one contribution of a GradJoin (ResNet identity).
    ``pool`` = (k, stride, pad): the output is max-pooled as well (ResNet stem); on GPU with ReLU the
    pool applies BN + ReLU to its window loads and the BN output is never stored.
    ``res_bn`` (act 'add_relu'): a BatchNorm2d module (act 'none') whose INPUT ``residual`` is; the
    residual added is res_bn(residual).  In training on GPU (bf16) it is applied inside the add's loads
    and its output is never stored (ResNet downsample branch)."""
    a = ACT[act]
    if res_bn is not None:
        m = res_bn
        if not (FUSE_RES_BN and BN_RELU_MASK and a == 2 and training and m.act == "none" and _native(z)
                and z.dtype == torch.bfloat16 and residual is not None and residual.dtype == torch.bfloat16
                and residual.shape == z.shape and z.shape[-1] % 8 == 0):
            residual = m(residual)
        else:
            rstate = (m.running_mean, m.running_var, m.num_batches_tracked.view(1), float(m.momentum), float(m.eps))
            out = BnActNHWC.apply(z.contiguous(), gamma, beta, residual.contiguous(), running_mean, running_var,
                                  num_batches_tracked, bool(training), float(momentum), float(eps), a, None, None,
                                  m.weight, m.bias, rstate)
            out._dpa_sum_on_load = out.requires_grad  # (as below: a deferred contribution is summed on load)
            return out
    if pool is not None:
        if not (FUSE_BN_POOL and a == 0 and _native(z) and z.shape[-1] % 8 == 0
                and z.dtype in (torch.float32, torch.bfloat16)):
            out = bn_act_nhwc(z, gamma, beta, running_mean, running_var, num_batches_tracked, training, momentum, eps,
                              act)
            return max_pool_nhwc(out, *pool)
        return BnActNHWC.apply(z.contiguous(), gamma, beta, None, running_mean, running_var, num_batches_tracked,
                               bool(training), float(momentum), float(eps), a, None, tuple(int(v) for v in pool))
    if a == 2 and residual is None:
        raise ValueError("act='add_relu' needs a residual")
    res = residual.to(z.dtype).contiguous() if residual is not None else None
    if res is not residual:
        res_join = None  # a converted copy: its gradient flows back through the conversion, not the join
    out = BnActNHWC.apply(z.contiguous(), gamma, beta, res, running_mean, running_var, num_batches_tracked,
                          bool(training), float(momentum), float(eps), a, res_join)
    # its backward sums a deferred second gradient contribution on load (GradJoin.defer)
    out._dpa_sum_on_load = bool(training) and out.requires_grad and _native(out)
    return out


class MaxPoolNHWC(torch.autograd.Function):
    """k x k / stride / pad max-pool on NHWC (fp32 or bf16) over csrc/kernels/pool.hip: the
    forward keeps a one-byte window position per output element, the backward gathers."""

    @staticmethod
    def forward(ctx, x, k: int, stride: int, pad: int):
        N, H, W, C = x.shape
        P, Q = conv_out(H, k, stride, pad), conv_out(W, k, stride, pad)
        y = torch.empty(N, P, Q, C, device=x.device, dtype=x.dtype)
        arg = torch.empty(N, P, Q, C, device=x.device, dtype=torch.uint8)
        _ext.require().maxpool_fwd(x, y, arg, k, stride, pad)
        ctx.save_for_backward(arg)
        ctx.geom = (N, H, W, C, k, stride, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        N, H, W, C, k, stride, pad = ctx.geom
        dx = torch.empty(N, H, W, C, device=dy.device, dtype=dy.dtype)
        _ext.require().maxpool_bwd(dy.contiguous(), arg, dx, k, stride, pad)
        return dx, None, None, None


def max_pool_nhwc(x: torch.Tensor, k: int = 3, stride: int = 2, pad: int = 1) -> torch.Tensor:
    """Max-pool on an NHWC tensor: the native kernels on GPU (C % 8 == 0), torch on CPU."""
    if _native(x) and x.shape[-1] % 8 == 0 and x.dtype in (torch.float32, torch.bfloat16):
        return MaxPoolNHWC.apply(x.contiguous(), int(k), int(stride), int(pad))
    y = F.max_pool2d(x.permute(0, 3, 1, 2), k, stride, pad)
    return y.permute(0, 2, 3, 1).contiguous()


def conv_out(h: int, k: int, stride: int, pad: int) -> int:
    return (h + 2 * pad - k) // stride + 1


def kaiming_uniform_krsc(K: int, R: int, S: int, C: int, c_true: Optional[int] = None) -> torch.Tensor:
    """torch's default Conv2d init (kaiming_uniform, a=sqrt(5)) in KRSC layout; channels beyond
    c_true (input padding) are zero."""
    c_true = c_true or C
    w = torch.empty(K, c_true, R, S)
    torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
    out = torch.zeros(K, R, S, C)
    out[..., :c_true] = w.permute(0, 2, 3, 1)
    return out


# ------------------------------------------------------------------ classifier head
def _gemm_splits(M: int, N: int, K: int) -> int:
    """Split-K count for gemm_f32.hip's 64x64 tiles: ~256 blocks, K chunks of at least 128."""
    tiles = -(-M // 64) * -(-N // 64)
    s = 1
    while tiles * s * 2 <= 256 and K // (s * 2) >= 128:
        s *= 2
    return s


_GEMM_SLAB = {}


def gemm_f32(a: torch.Tensor, b: torch.Tensor, trans_a: bool = False, trans_b: bool = False,
             bias: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = op(a) @ op(b) (+ bias) in exact fp32 on the matrix cores (gemm_f32.hip); op = transpose
    when the flag is set.  Split-K workspace cached per device."""
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    N = b.shape[0] if trans_b else b.shape[1]
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=torch.float32)
    s = _gemm_splits(M, N, K) if (M * N) % 4 == 0 else 1
    slab = None
    if s > 1:
        slab = _GEMM_SLAB.get(a.device)
        if slab is None or slab.numel() < s * M * N:
            slab = _GEMM_SLAB[a.device] = torch.empty(s * M * N, device=a.device, dtype=torch.float32)
    _ext.require().gemm_f32(a, b, out, trans_a, trans_b, bias, s, slab)
    return out


def _head_fwd(x, weight, bias):
    """feat = GAP(x) fp32 [N,C] (head.hip), logits = feat @ W^T + b (gemm_f32.hip)."""
    if not _native(x):  # CPU oracle path
        feat = x.to(weight.dtype).mean(dim=(1, 2))
        return feat, torch.addmm(bias, feat, weight.t())
    feat = torch.empty(x.shape[0], x.shape[-1], device=x.device, dtype=torch.float32)
    _ext.require().gap(x, feat)
    return feat, gemm_f32(feat, weight, trans_b=True, bias=bias)


def _head_bwd(dlogits, gscale, feat, weight, wparam, bparam, shape, dtype):
    """Gradients of GAP + Linear from dlogits * gscale (gscale: 1-element device tensor): db and dW
    straight into the optimizer arena when the DDP wrapper offers slots."""
    N, H, W, C = shape
    if not _native(feat):
        dl = dlogits * gscale
        dfeat = dl @ weight
        dx = (dfeat / (H * W))[:, None, None, :].expand(N, H, W, C).to(dtype).contiguous()
        dw, db = dl.t() @ feat, dl.sum(0)
        sw, sb = grad_slot(wparam), grad_slot(bparam)
        if sw is not None:
            dw = sw.copy_(dw)
        if sb is not None:
            db = sb.copy_(db)
        return dx, dw, db
    K = _ext.require()
    dev = feat.device
    dl = torch.empty_like(dlogits)
    db = grad_slot(bparam)
    if db is None:
        db = torch.empty(weight.shape[0], device=dev, dtype=torch.float32)
    K.head_bwd_prep(dlogits, gscale, dl, db)  # dl = dlogits * g, db = column sums (fixed order)
    dfeat = gemm_f32(dl, weight)
    dw = grad_slot(wparam)
    if dw is None:
        dw = torch.empty_like(weight)
    gemm_f32(dl, feat, trans_a=True, out=dw)
    dx = torch.empty(shape, device=dev, dtype=dtype)
    K.gap_bwd(dfeat, dx)
    return dx, dw, db


class HeadLinear(torch.autograd.Function):
    """logits = Linear(GAP(x)): global average pool (head.hip) + fp32 MFMA GEMM (gemm_f32.hip), one
    autograd node."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        note_use(weight)
        note_use(bias)
        feat, logits = _head_fwd(x, weight, bias)
        ctx.save_for_backward(feat, weight)
        ctx.w_b, ctx.x_meta = (weight, bias), (x.shape, x.dtype)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        feat, weight = ctx.saved_tensors
        one = torch.ones(1, device=feat.device, dtype=feat.dtype)
        dx, dw, db = _head_bwd(dlogits.contiguous().to(feat.dtype), one, feat, weight, *ctx.w_b, *ctx.x_meta)
        return dx, dw, db


class HeadCE(torch.autograd.Function):
    """Global average pool + Linear + softmax cross-entropy (mean) in one autograd node
    (csrc/kernels/head.hip; the three GEMMs on the fp32 matrix cores, gemm_f32.hip).  The loss
    gradient is formed in the forward (as the VGG head does, fc_ce.hip); the backward scales it by
    the incoming gradient, reduces the bias gradient, and writes weight / bias gradients straight
    into the optimizer arena when the DDP wrapper offers a slot (``grad_slot``)."""

    @staticmethod
    def forward(ctx, x, weight, bias, target):
        N = x.shape[0]
        note_use(weight)
        note_use(bias)
        feat, logits = _head_fwd(x, weight, bias)
        if not _native(x):
            loss = F.cross_entropy(logits, target)
            p = torch.softmax(logits, 1)
            p[torch.arange(N), target] -= 1.0
            dlogits = p / N
        else:
            dev = x.device
            loss_row = torch.empty(N, device=dev, dtype=torch.float32)
            dlogits = torch.empty_like(logits)
            loss = torch.empty((), device=dev, dtype=torch.float32)
            _ext.require().softmax_ce(logits, target, loss_row, dlogits, None, loss.view(1), None)
        ctx.save_for_backward(feat, dlogits, weight)
        ctx.w_b, ctx.x_meta = (weight, bias), (x.shape, x.dtype)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        feat, dlogits, weight = ctx.saved_tensors
        g = gloss.reshape(1).to(dtype=feat.dtype).contiguous()
        dx, dw, db = _head_bwd(dlogits, g, feat, weight, *ctx.w_b, *ctx.x_meta)
        return dx, dw, db, None


def head_ce(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Batch-mean cross-entropy of Linear(GAP(x)) (x NHWC bf16/fp32; weight [J,C], bias [J] fp32)."""
    return HeadCE.apply(x.contiguous(), weight, bias, target.contiguous())


def head_logits(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """Linear(GAP(x)) logits, differentiable (for callers that apply their own loss)."""
    return HeadLinear.apply(x.contiguous(), weight, bias)
