"""Tracing hooks (new scope: the reference only has datetime deltas — SURVEY §5.1).

* ``trace_range(name)`` — a roctx range (via torch's ROCm-built nvtx bindings, which emit
  roctx) around fwd / bwd / sync / step, visible in ``rocprofv3 --marker-trace``.  No-op on CPU.
* ``StepTimer`` — HIP-event timing of phases (GPU work is asynchronous; host timestamps only
  measure launch time unless synchronised).
* ``debug_sync`` — when ``DPA_DEBUG_SYNC=1`` every collective region is followed by a full
  device synchronize (race-detection aid for comm/compute stream ordering).
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, List

import torch

_ENABLED = os.environ.get("DPA_TRACE", "0") == "1"
DEBUG_SYNC = os.environ.get("DPA_DEBUG_SYNC", "0") == "1"


def enable_tracing(on: bool = True):
    global _ENABLED
    _ENABLED = on


@contextlib.contextmanager
def trace_range(name: str):
    if _ENABLED and torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)
            pushed = True
        except Exception:
            pushed = False
        try:
            yield
        finally:
            if pushed:
                torch.cuda.nvtx.range_pop()
    else:
        yield


class StepTimer:
    """Accumulates per-phase GPU time with HIP events; ``summary()`` syncs once."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.on = self.device.type == "cuda"
        self._marks: List[tuple] = []

    def mark(self, name: str):
        if not self.on:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self._marks.append((name, e))

    def summary(self) -> Dict[str, float]:
        if not self.on or len(self._marks) < 2:
            return {}
        torch.cuda.synchronize(self.device)
        out: Dict[str, float] = {}
        for (n0, e0), (n1, e1) in zip(self._marks, self._marks[1:]):
            out[n1] = out.get(n1, 0.0) + e0.elapsed_time(e1)
        self._marks.clear()
        return out
