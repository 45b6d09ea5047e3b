"""Tracing and step-timing hooks (new scope: the reference only has datetime deltas, main.py:31,38-39;
SURVEY §5.1).

* ``trace_range(name)`` — a roctx range (torch's ROCm-built nvtx bindings emit roctx) around
  fwd / bwd / sync / step, visible in ``rocprofv3 --marker-trace``.  No-op on CPU.
* ``EventProbe`` — timing HIP events recorded on the stream that is current at each mark (compute,
  wgrad or comm stream), read back once per step.  GPU work is asynchronous, so phase times have to
  come from the device clock.  The benches use it in a short diagnostic phase after the timed
  steps (timing events carry a system-scope fence, so they are kept out of the timed region) to
  report the communication left exposed after backward and each bucket's collective time.
* ``rocprof_command(argv)`` — the ``rocprofv3 --kernel-trace --stats`` command line that profiles
  a run of this program (the program itself goes right after ``--``: no env/bash hop, which the
  profiler's preloaded library would turn into an exec of a GPU-initialised process).
"""
from __future__ import annotations

import contextlib
import os
import shlex
import sys
from typing import Dict, List, Optional, Sequence, Tuple

import torch

_ENABLED = os.environ.get("DPA_TRACE", "0") == "1"


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


class EventProbe:
    """Named timing events on whatever stream is current at ``mark``; ``times()`` synchronises
    once and returns every mark's time in ms relative to the first mark."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.on = self.device.type == "cuda"
        self._marks: List[Tuple[str, torch.cuda.Event]] = []

    def reset(self):
        self._marks.clear()

    def mark(self, name: str):
        if not self.on:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream(self.device))
        self._marks.append((name, e))

    def times(self) -> Dict[str, float]:
        if not self.on or not self._marks:
            return {}
        torch.cuda.synchronize(self.device)
        t0 = self._marks[0][1]
        return {n: t0.elapsed_time(e) for n, e in self._marks}


def step_comm_report(samples: Sequence[Dict[str, float]], nbuckets: int) -> Dict[str, object]:
    """Aggregate per-step EventProbe readings (marks ``bwd_end``, ``synced``, ``step_end`` and
    ``b{i}_start`` / ``b{i}_end`` per bucket) into medians: the exposed communication after backward
    (``synced - bwd_end``: the compute stream waiting for the comm stream), and per bucket the
    collective's duration and its end relative to the end of backward."""
    def med(v: List[float]) -> Optional[float]:
        v = sorted(x for x in v if x is not None)
        return round(v[len(v) // 2], 4) if v else None

    out: Dict[str, object] = {
        "exposed_comm_ms": med([s["synced"] - s["bwd_end"] for s in samples if "synced" in s and "bwd_end" in s]),
        "bwd_ms": med([s["bwd_end"] for s in samples if "bwd_end" in s]),
        "step_ms": med([s["step_end"] for s in samples if "step_end" in s]),
    }
    buckets = []
    for i in range(nbuckets):
        d = [s[f"b{i}_end"] - s[f"b{i}_start"] for s in samples if f"b{i}_end" in s and f"b{i}_start" in s]
        e = [s[f"b{i}_end"] - s["bwd_end"] for s in samples if f"b{i}_end" in s and "bwd_end" in s]
        if d:
            buckets.append({"coll_ms": med(d), "end_after_bwd_ms": med(e)})
    out["buckets"] = buckets
    return out


def rocprof_command(argv: Sequence[str], outdir: str = "gpurun_out/prof", python: Optional[str] = None) -> List[str]:
    """``rocprofv3 --kernel-trace --stats -d outdir -o run --output-format csv -- python3 <argv>``."""
    py = python or sys.executable
    return ["rocprofv3", "--kernel-trace", "--stats", "-d", outdir, "-o", "run", "--output-format", "csv", "--",
            py, *argv]


def format_command(cmd: Sequence[str]) -> str:
    return " ".join(shlex.quote(c) for c in cmd)
