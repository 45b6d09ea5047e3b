"""Shared plumbing of the benches (bench.py, bench_resnet.py).

* ``relaunch``: ``--profile`` re-runs the program under ``rocprofv3 --kernel-trace --stats`` as a
  child; ``--gpus N`` started without a launcher environment starts N local ranks
  (parallel/spawn.py).  Both happen before anything touches the GPU, and the parent only waits
  for its children and exits with their code.
* ``timed_steps``: W untimed warmup steps, then K steps bracketed by a device synchronize + barrier
  on both sides; the elapsed time is the max over ranks.
* ``replicas_max_diff``: element-wise max|max_r p - min_r p| of a parameter arena over all ranks
  (0.0 ⇔ every replica holds bitwise identical parameters).
"""
from __future__ import annotations

import os
import subprocess
import sys
import time
from typing import Callable, List, Optional, Sequence

import torch

from ..parallel.spawn import is_spawned_child, launch, needs_spawn
from .profiling import format_command, rocprof_command

PROFILED_ENV = "DPA_PROFILED"


def strip_flag(argv: Sequence[str], flag: str, takes_value: bool = False) -> List[str]:
    out, skip = [], False
    for i, a in enumerate(argv):
        if skip:
            skip = False
            continue
        if a == flag:
            skip = takes_value
            continue
        if takes_value and a.startswith(flag + "="):
            continue
        out.append(a)
    return out


def relaunch(script: str, argv: Sequence[str], gpus: int, profile: bool, profile_dir: str,
             timeout_s: float) -> Optional[int]:
    """Return an exit code if this process only supervised children, else None (run here)."""
    if profile and os.environ.get(PROFILED_ENV) != "1" and not is_spawned_child():
        child_argv = [script] + strip_flag(argv, "--profile")
        cmd = rocprof_command(child_argv, outdir=profile_dir)
        print(f"[profile] {format_command(cmd)}", file=sys.stderr, flush=True)
        env = dict(os.environ, **{PROFILED_ENV: "1"})
        return subprocess.call(cmd, env=env)
    if needs_spawn(gpus):
        return launch(script, list(argv), gpus, timeout_s=timeout_s)
    return None


def device_barrier(ctx, dev: torch.device):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    ctx.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def timed_steps(step: Callable[[], None], steps: int, warmup: int, ctx, dev: torch.device) -> float:
    """Seconds for ``steps`` steps after ``warmup`` untimed ones; max over ranks."""
    for _ in range(warmup):
        step()
    device_barrier(ctx, dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    device_barrier(ctx, dev)
    el = time.perf_counter() - t0
    return ctx.all_max(el)


@torch.no_grad()
def replicas_max_diff(comm, flat: torch.Tensor) -> float:
    if comm.world <= 1:
        return 0.0
    mx, mn = flat.clone(), flat.clone()
    with comm.region():
        comm.all_reduce(mx, "max")
        comm.all_reduce(mn, "min")
    comm.wait()
    return float((mx - mn).abs().max().item())


def comm_world(comm) -> Optional[int]:
    """Ranks an RCCL communicator itself reports (ncclCommCount); None when the run has no RCCL
    communicator (null comm of a 1-GPU run, torch/gloo process groups)."""
    f = getattr(comm, "comm_count", None)
    return int(f()) if f is not None else None


def torch_eager_baseline(steps: int, warmup: int, batch: int, timeout_s: float = 300.0) -> Optional[dict]:
    """Stock PyTorch-ROCm eager fp32 VGG-11 step (tools/torch_baseline.py: MIOpen convs, torch SGD)
    timed in a CHILD process on this run's GPU, before this process touches the device.  Returns
    its JSON record, or None if it failed."""
    import json

    tool = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools",
                        "torch_baseline.py")
    cmd = [sys.executable, tool, "--steps", str(steps), "--warmup", str(warmup), "--batch", str(batch),
           "--modes", "fp32"]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return None
    if r.returncode != 0:
        return None
    for line in reversed(r.stdout.strip().splitlines()):
        try:
            return json.loads(line)
        except ValueError:
            continue
    return None
