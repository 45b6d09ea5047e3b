"""NHWC ``nn.Module`` layers over the autograd kernels (ops/functional.py).

Weights live in the kernels' layout (conv KRSC, input channels padded to a multiple of 8) and are
converted at the ``state_dict`` boundary, so checkpoints keep torch's OIHW keys/shapes and load
into / from the stock torch modules of the same architecture.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import functional as Fn


def _pad8(c: int) -> int:
    return (c + 7) // 8 * 8


class Conv2d(nn.Module):
    """Bias-free NHWC conv (every conv in the supported models feeds a BatchNorm)."""

    def __init__(self, cin: int, cout: int, k: int, stride: int = 1, padding: int = 0, impl: str = "bf16"):
        super().__init__()
        self.cin, self.cout, self.k, self.stride, self.padding, self.impl = cin, cout, k, stride, padding, impl
        self.cin_pad = _pad8(cin)
        self.weight = nn.Parameter(Fn.kaiming_uniform_krsc(cout, k, k, self.cin_pad, cin))
        self.weight._dpa_direct = True  # the conv backward can write its gradient into an optimizer slot
        self._register_state_dict_hook(Conv2d._to_oihw)
        self._register_load_state_dict_pre_hook(self._from_oihw)

    def forward(self, x, join=None):
        # a network input with fewer channels than cin_pad is zero-padded inside the op (on GPU in
        # the bf16 plane split, pad_split8: no padded copy of the input)
        return Fn.conv2d_nhwc(x, self.weight, self.stride, self.padding, self.impl, join)

    @staticmethod
    def _to_oihw(module, sd, prefix, local_metadata):
        w = sd[prefix + "weight"]
        sd[prefix + "weight"] = w[..., :module.cin].permute(0, 3, 1, 2).contiguous()
        return sd

    def _from_oihw(self, sd, prefix, *args):
        key = prefix + "weight"
        if key in sd and sd[key].dim() == 4 and sd[key].shape[1] == self.cin and sd[key].shape[-1] == self.k \
                and tuple(sd[key].shape) != tuple(self.weight.shape):
            w = sd[key]
            out = torch.zeros(self.cout, self.k, self.k, self.cin_pad, dtype=w.dtype, device=w.device)
            out[..., :self.cin] = w.permute(0, 2, 3, 1)
            sd[key] = out

    def extra_repr(self):
        return f"{self.cin}, {self.cout}, k={self.k}, stride={self.stride}, padding={self.padding}, impl={self.impl}"


class BatchNorm2d(nn.Module):
    """BatchNorm2d (torch semantics: momentum, unbiased running var, num_batches_tracked) fused
    with its activation: ``act`` in {"relu", "none", "add_relu"} (the last takes a residual)."""

    def __init__(self, c: int, act: str = "relu", momentum: float = 0.1, eps: float = 1e-5):
        super().__init__()
        self.c, self.act, self.momentum, self.eps = c, act, momentum, eps
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.weight._dpa_direct = self.bias._dpa_direct = True  # BN backward writes into optimizer slots
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))

    def forward(self, z, residual=None, res_join=None, pool=None, res_bn=None):
        """``pool`` = (k, stride, pad): also max-pool the output; ``res_bn``: ``residual`` is the input of
        that BatchNorm2d module (fused on GPU, see Fn.bn_act_nhwc)."""
        nbt = self.num_batches_tracked.view(1) if self.training else None
        return Fn.bn_act_nhwc(z, self.weight, self.bias, self.running_mean, self.running_var, nbt, self.training,
                              self.momentum, self.eps, self.act, residual, res_join, pool, res_bn)

    def extra_repr(self):
        return f"{self.c}, act={self.act}"


class MaxPool2d(nn.Module):
    def __init__(self, k: int = 3, stride: int = 2, padding: int = 1):
        super().__init__()
        self.k, self.stride, self.padding = k, stride, padding

    def forward(self, x):
        return Fn.max_pool_nhwc(x, self.k, self.stride, self.padding)
