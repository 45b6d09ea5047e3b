"""Cross-stream dependencies between the compute, wgrad and comm HIP streams of one GPU.

``torch.cuda.Event`` records with a system-scope release: every record writes back and
invalidates L2, and the next kernel on the recording stream starts only after that (measured with
``tools/event_overhead.py``).  The step's dependencies are all between streams of one device, so
the framework records native events (``_C.DevEvent``) with a device-scope release instead.

(hipEventReleaseToDevice; torch events and hipEventDisableSystemFence were measured slower,
docs/PERF_NOTES.md.)
"""
from __future__ import annotations

from typing import Optional

import torch

def _native_flags() -> Optional[int]:
    from .. import _ext

    C = _ext.require()
    return C.EVENT_DISABLE_TIMING | C.EVENT_RELEASE_TO_DEVICE


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
