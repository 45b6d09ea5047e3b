"""Generic bucketed data parallelism for any ``nn.Module`` (the hook-based path; the VGG engine
uses the static schedule in sync.py).  Semantics follow torch ``DistributedDataParallel`` as the
reference uses it (main_ddp.py:137): rank 0's parameters and buffers are broadcast at wrap time,
floating buffers (BN running stats) and counters are broadcast before every training forward,
gradients are summed over ranks in buckets while backward is still running and scaled by 1/W.

MI355X-first mechanics instead of torch's Reducer:
* parameters and gradients are re-homed into two flat arenas laid out in REVERSE registration
  order (~ gradient-ready order), so every bucket is one contiguous slice — no copy into / out of
  bucket buffers (``mul_out`` / ``copy_bucket_to_grad``) and the optimizer is one fused kernel
  (``FlatSGD``);
* ``register_post_accumulate_grad_hook`` marks tensors ready; a bucket's all-reduce is issued on
  the communicator's stream (RCCL over xGMI) as soon as its last gradient lands;
* ``finish()`` issues any remainder, makes the compute stream wait, and returns the 1/W scale that
  ``FlatSGD.step`` folds into the update (no separate scaling pass).
Gradients are accumulated in place into the arena views, so ``zero_grad`` must keep them
(``FlatSGD.zero_grad`` / ``DistributedDataParallel.zero_grad`` memset the arena).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.nn as nn

from ..ops.functional import NPLANES
from .comm import Comm, NullComm

ALIGN = 64


class _Flat:
    """Tensors re-homed as views of one contiguous buffer (64-element aligned entries)."""

    def __init__(self, tensors: List[torch.Tensor], dtype, device):
        self.offsets, off = [], 0
        for t in tensors:
            self.offsets.append(off)
            off += (t.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.flat = torch.zeros(max(off, ALIGN), dtype=dtype, device=device)
        self.numel = off

    def view(self, i: int, t: torch.Tensor) -> torch.Tensor:
        o = self.offsets[i]
        return self.flat[o:o + t.numel()].view_as(t)


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, comm: Optional[Comm] = None, bucket_mb: float = 25.0,
                 broadcast_buffers: bool = True, overlap: bool = True):
        super().__init__()
        self.module = module
        self.comm = comm or NullComm()
        self.world = self.comm.world
        self.active = self.comm.name != "null"
        self.broadcast_buffers = broadcast_buffers
        self.overlap = overlap
        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise ValueError("module has no trainable parameters")
        dev, dt = params[0].device, params[0].dtype
        order = list(reversed(params))  # ~ gradient-ready order
        self._params = order
        self._pflat = _Flat(order, dt, dev)
        self._gflat = _Flat(order, dt, dev)
        # parameters whose producing kernel writes its gradient straight into the arena slot (conv
        # weights, BN affine: ops/functional.grad_slot) keep p.grad = None until backward hands
        # autograd the arena view; the rest accumulate into a pre-assigned arena view
        self._direct = [bool(getattr(p, "_dpa_direct", False)) for p in order]
        with torch.no_grad():
            for i, p in enumerate(order):
                v = self._pflat.view(i, p)
                v.copy_(p.data)
                p.data = v
                if self._direct[i]:
                    p._dpa_grad_slot = (lambda i=i, p=p: self._gflat.view(i, p))
                    p.grad = None
                else:
                    p.grad = self._gflat.view(i, p)
        # buckets: contiguous arena slices of ~bucket_mb, cut at tensor boundaries
        cap = max(1, int(bucket_mb * (1 << 20) / self._gflat.flat.element_size()))
        self._buckets: List[List[int]] = []
        cur, cur_n = [], 0
        for i, p in enumerate(order):
            n = (p.numel() + ALIGN - 1) // ALIGN * ALIGN
            if cur and cur_n + n > cap:
                self._buckets.append(cur)
                cur, cur_n = [], 0
            cur.append(i)
            cur_n += n
        if cur:
            self._buckets.append(cur)
        self._bucket_of = {i: b for b, idx in enumerate(self._buckets) for i in idx}
        self._pending: List[int] = []
        self._issued: List[bool] = []
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i)) for i, p in enumerate(order)]
        # buffers: floating ones (BN running stats) in one arena, integer counters in another
        fb = [b for b in module.buffers() if b.is_floating_point()]
        ib = [b for b in module.buffers() if not b.is_floating_point()]
        self._bufs = []
        for group, dtype in ((fb, dt), (ib, torch.int64)):
            if not group:
                continue
            fl = _Flat(group, dtype, dev)
            with torch.no_grad():
                for i, b in enumerate(group):
                    v = fl.view(i, b)
                    v.copy_(b.data)
                    b.data = v
            self._bufs.append(fl)
        self._reset()
        self._bufs_sent = False   # buffers broadcast during the current step (first gradient hook)
        self._bufs_fresh = False  # replicas already hold rank 0's buffers for the next forward
        if self.active:
            self.comm.prepare([self._gflat.flat, self._pflat.flat] + [fl.flat for fl in self._bufs])
            self._broadcast_state()
        self._init_planes(order, dev)

    def _init_planes(self, order, dev):
        """bf16 operand planes of the conv weights, kept current by the fused SGD kernel (one
        split per update instead of one per conv call): [NP, arena] bf16, each conv weight reads
        its slice (ops/functional.weight_planes)."""
        self._planes = None
        convs = [m for m in self.module.modules() if hasattr(m, "impl") and hasattr(m, "cin_pad")]
        nps = {NPLANES.get(m.impl) for m in convs}
        if dev.type != "cuda" or len(nps) != 1 or None in nps or self._pflat.flat.dtype != torch.float32:
            return
        np_ = nps.pop()
        from .. import _ext

        self._planes = torch.empty(np_, self._pflat.flat.numel(), dtype=torch.bfloat16, device=dev)
        _ext.require().split_planes(self._pflat.flat, self._planes)
        conv_w = {id(m.weight) for m in convs}
        for i, p in enumerate(order):
            if id(p) in conv_w:
                o = self._pflat.offsets[i]
                p._dpa_planes = self._planes[:, o:o + p.numel()].view((np_,) + tuple(p.shape))
                p._dpa_planes_ver = p._version

    @property
    def weight_planes(self) -> Optional[torch.Tensor]:
        return self._planes

    # ---------------------------------------------------------------- state sync
    def _broadcast_state(self):
        with self.comm.region():
            self.comm.broadcast(self._pflat.flat, 0)
            for fl in self._bufs:
                self.comm.broadcast(fl.flat, 0)
        self.comm.wait()

    def _reset(self):
        self._pending = [len(b) for b in self._buckets]
        self._issued = [False] * len(self._buckets)
        self._seen = [False] * len(self._params)

    def _send_buffers(self):
        with self.comm.region():
            for fl in self._bufs:
                self.comm.broadcast(fl.flat, 0)

    def forward(self, *args, **kwargs):
        self._reset()
        for p in self._params:
            p._dpa_uses = 0
        if self.active and self.broadcast_buffers and self._bufs and self.module.training:
            if self._bufs_fresh:  # broadcast right after the previous training forward
                self._bufs_fresh = False
            else:
                self._send_buffers()
                self.comm.wait()
        self._bufs_sent = False
        return self.module(*args, **kwargs)

    # ---------------------------------------------------------------- gradient buckets
    def _make_hook(self, i: int):
        def hook(p):
            self._seen[i] = True
            if self._direct[i]:
                # a parameter used more than once in the forward gets its gradient summed by
                # autograd into a fresh tensor: move it into the arena slot the collectives and the
                # fused optimizer read
                v = self._gflat.view(i, p)
                if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                    with torch.no_grad():
                        v.copy_(p.grad)
                    p.grad = v
            # first gradient of the step: the forward is over, so rank 0's buffers (BN running
            # stats) are final for this step -- broadcast them now, under the backward, instead of
            # before the next forward (nothing changes them in between; finish() orders the
            # compute stream after the comm stream)
            if not self._bufs_sent and self.active and self.broadcast_buffers and self._bufs \
                    and self.module.training:
                self._send_buffers()
                self._bufs_sent = self._bufs_fresh = True
            b = self._bucket_of[i]
            self._pending[b] -= 1
            if self._pending[b] == 0 and self.overlap:
                self._issue(b)
        return hook

    def _span(self, b: int):
        idx = self._buckets[b]
        lo = self._gflat.offsets[idx[0]]
        last = idx[-1]
        hi = self._gflat.offsets[last] + (self._params[last].numel() + ALIGN - 1) // ALIGN * ALIGN
        return lo, hi

    def _issue(self, b: int):
        if self._issued[b] or not self.active:
            self._issued[b] = True
            return
        self._issued[b] = True
        lo, hi = self._span(b)
        with self.comm.region():
            self.comm.all_reduce(self._gflat.flat[lo:hi], "sum")

    def finish(self) -> float:
        """After backward: issue what is left, order the compute stream after the collectives and
        return the gradient scale (1/W) for the optimizer."""
        for i, (p, d) in enumerate(zip(self._params, self._direct)):
            if d and not self._seen[i]:  # a slot-written parameter that got no gradient this step
                with torch.no_grad():
                    self._gflat.view(i, p).zero_()
        for b in range(len(self._buckets)):
            if not self._issued[b]:
                self._issue(b)
        if self.active:
            self.comm.wait()
        return 1.0 / self.world

    def zero_grad(self, set_to_none: bool = False):
        """Parameters whose backward writes their arena slot (``_dpa_direct``: every conv / BN / head
        parameter of the kernel layers) need no memset -- the slot is overwritten, and finish() zeroes
        the slot of any that got no gradient; the others accumulate into their view, which is zeroed."""
        with torch.no_grad():
            for i, (p, d) in enumerate(zip(self._params, self._direct)):
                if d:
                    p.grad = None  # backward hands autograd the arena view again
                else:
                    self._gflat.view(i, p).zero_()

    @property
    def flat_params(self) -> torch.Tensor:
        return self._pflat.flat

    @property
    def flat_grads(self) -> torch.Tensor:
        return self._gflat.flat

    def num_buckets(self) -> int:
        return len(self._buckets)


class FlatSGD:
    """torch.optim.SGD semantics (momentum, dampening 0, weight decay, no nesterov) as ONE fused
    kernel over the DDP arenas; ``step(grad_scale)`` folds the 1/W DDP scale in."""

    def __init__(self, ddp: DistributedDataParallel, lr: float, momentum: float = 0.0, weight_decay: float = 0.0):
        self.ddp = ddp
        self.lr, self.momentum, self.weight_decay = lr, momentum, weight_decay
        self.buf = torch.zeros_like(ddp.flat_params)
        self.steps = 0

    def zero_grad(self, set_to_none: bool = False):
        self.ddp.zero_grad()

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0):
        p, g = self.ddp.flat_params, self.ddp.flat_grads
        if p.is_cuda:
            from .. import _ext

            _ext.require().sgd_flat(p, g, self.buf, self.lr, self.momentum, self.weight_decay, grad_scale,
                                    self.steps == 0, 0, -1, self.ddp.weight_planes)
        else:
            from ..ops import cpu_ref

            cpu_ref.sgd_flat(p, g, self.buf, self.lr, self.momentum, self.weight_decay, grad_scale, self.steps == 0)
        self.steps += 1
