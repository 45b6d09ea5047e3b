"""Cross-stream dependencies between the compute, wgrad and comm HIP streams of one GPU.

Events record with the default (system-scope) release.  Rounds 2-4 recorded them with a
device-scope release (hipEventReleaseToDevice: no L2 writeback at the record), measured neutral
to +1 % at the time.  Round 5 found it unsafe on MI355X: with four ranks sharing one GPU through the
peer-memory collectives, ~30 % of runs computed the first layer of a step from partly stale input
(15-17 of conv0's 256 workgroups produced different output for the same input and weights,
after the compute stream had waited on a device-scope event of the comm stream); with system-scope
events 10 of 10 runs were bitwise identical, at the same speed (1 GPU: 222.4k vs 222.3k img/s, 1-rank
RCCL: 217.9k vs 217.8k; docs/PERF_NOTES.md round 5).
"""
from __future__ import annotations

from typing import Optional

import torch


def _native_flags() -> Optional[int]:
    from .. import _ext

    return _ext.require().EVENT_DISABLE_TIMING


class DevEvent:
    """A reusable dependency event: ``record(stream)`` on the producer, ``wait(stream)`` on the
    consumer (the wait captures the latest record, as with CUDA/HIP events)."""

    __slots__ = ("_ev", "_native")

    def __init__(self):
        flags = _native_flags()
        if flags is None:
            self._ev, self._native = torch.cuda.Event(), False
        else:
            from .. import _ext

            self._ev, self._native = _ext.require().DevEvent(flags), True

    def record(self, stream: Optional[torch.cuda.Stream] = None):
        stream = stream if stream is not None else torch.cuda.current_stream()
        if self._native:
            self._ev.record(stream.cuda_stream)
        else:
            self._ev.record(stream)

    def wait(self, stream: Optional[torch.cuda.Stream] = None):
        stream = stream if stream is not None else torch.cuda.current_stream()
        if self._native:
            self._ev.wait(stream.cuda_stream)
        else:
            stream.wait_event(self._ev)

    def synchronize(self):
        self._ev.synchronize()


class StreamJoin:
    """``consumer`` waits for everything queued so far on ``producer`` (torch's
    ``Stream.wait_stream`` with a device-scope event reused across calls)."""

    __slots__ = ("_ev",)

    def __init__(self):
        self._ev = DevEvent()

    def __call__(self, consumer: torch.cuda.Stream, producer: torch.cuda.Stream):
        if consumer == producer:
            return
        self._ev.record(producer)
        self._ev.wait(consumer)
