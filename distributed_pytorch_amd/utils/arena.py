"""Flat arenas: many named tensors packed into ONE contiguous buffer.

Parameters, gradients and momentum live in three arenas with identical layouts, so the fused
SGD kernel is one launch over the whole model, DDP buckets are plain contiguous slices (no
``copy_bucket_to_grad``), and gather/broadcast move one buffer (SURVEY §7.1 "Flat parameter/grad
arenas").  Each entry starts on a 64-element (256 B) boundary so every view is float4-aligned.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Iterable, List, Tuple

import torch

ALIGN = 64


class Arena:
    def __init__(self, entries: Iterable[Tuple[str, Tuple[int, ...]]], device, dtype=torch.float32, align=ALIGN):
        self.shapes: "OrderedDict[str, Tuple[int, ...]]" = OrderedDict()
        self.offsets: Dict[str, int] = {}
        self.numels: Dict[str, int] = {}
        off = 0
        for name, shape in entries:
            n = 1
            for s in shape:
                n *= int(s)
            self.shapes[name] = tuple(int(s) for s in shape)
            self.offsets[name] = off
            self.numels[name] = n
            off += (n + align - 1) // align * align
        self.numel = off
        self.device = torch.device(device)
        self.dtype = dtype
        self.flat = torch.zeros(max(off, align), device=device, dtype=dtype)
        self.views: "OrderedDict[str, torch.Tensor]" = OrderedDict(
            (k, self.flat[self.offsets[k]:self.offsets[k] + self.numels[k]].view(self.shapes[k])) for k in self.shapes)

    def like(self) -> "Arena":
        """A zero-initialised arena with the same layout."""
        return Arena(self.shapes.items(), self.device, self.dtype)

    def names(self) -> List[str]:
        return list(self.shapes.keys())

    def span(self, names: Iterable[str]) -> Tuple[int, int]:
        """[start, end) element range covering the given (adjacent) entries, padded ends included."""
        names = list(names)
        lo = min(self.offsets[n] for n in names)
        hi = max(self.offsets[n] + (self.numels[n] + ALIGN - 1) // ALIGN * ALIGN for n in names)
        return lo, hi

    def __getitem__(self, name: str) -> torch.Tensor:
        return self.views[name]

    def __contains__(self, name: str) -> bool:
        return name in self.views
