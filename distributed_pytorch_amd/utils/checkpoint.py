"""Per-rank checkpoint / resume (new scope: the reference has none — SURVEY §5.4).

Layout: ``<dir>/rank{R}.pt`` holding

    {"model": reference-layout state_dict (58 keys for VGG-11, OIHW fp32; "module." prefix when
               saved from DDP mode, as DistributedDataParallel.state_dict() would),
     "optimizer": torch.optim.SGD state_dict (momentum_buffer per param),
     "epoch": int, "batch_idx": int (next batch to run), "sampler_seed": int,
     "world": int, "mode": str, "steps_taken": int, "rng": torch CPU RNG state}

``model`` loads straight into ``model.VGG11().load_state_dict`` (after stripping ``module.``).
Loading uses ``torch.load(weights_only=True)`` — nothing in the file is executed.

Resume safety:
* a checkpoint written by a run with a different world size or sync mode is refused (its
  ``batch_idx`` indexes a different shard); ``reshard=True`` (``--resume-reshard``) loads the
  weights and optimizer state anyway and restarts the saved epoch at batch 0.  A rank with no file
  of its own (the world grew: ranks >= the old world size) then loads the lowest-numbered rank's
  file — after ``prepare_checkpoint`` every rank saved identical parameters and full momentum;
* ``agree`` (after every rank loaded) checks that all ranks resume from the same
  (epoch, batch_idx, steps_taken) — ranks holding checkpoints of different iterations (a crash
  between two ``--checkpoint-every`` writes) or a rank without one would otherwise pair gradients
  of different steps in same-shaped collectives.
"""
from __future__ import annotations

import os
import warnings
from typing import Optional, Tuple

import torch


class ResumeMismatch(RuntimeError):
    pass


def path_for(ckpt_dir: str, rank: int) -> str:
    return os.path.join(ckpt_dir, f"rank{rank}.pt")


def save(ckpt_dir: str, rank: int, engine, epoch: int, batch_idx: int, sampler_seed: int = 0, world: int = 1,
         mode: str = "single", ddp_prefix: bool = False) -> str:
    os.makedirs(ckpt_dir, exist_ok=True)
    obj = {
        "model": engine.state_dict(prefix="module." if ddp_prefix else ""),
        "optimizer": engine.optimizer_state_dict(),
        "epoch": int(epoch),
        "batch_idx": int(batch_idx),
        "sampler_seed": int(sampler_seed),
        "world": int(world),
        "mode": mode,
        "steps_taken": int(engine.steps_taken),
        "rng": torch.get_rng_state(),
    }
    p = path_for(ckpt_dir, rank)
    tmp = p + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, p)
    return p


def load(ckpt_dir: str, rank: int, engine, map_location="cpu", world: Optional[int] = None,
         mode: Optional[str] = None, reshard: bool = False) -> Optional[dict]:
    """Load rank's checkpoint into ``engine``; returns the checkpoint dict (with ``batch_idx``
    reset to 0 when resharding) or None if there is none.  ``world`` / ``mode``: the current run's,
    validated against the saved ones."""
    p = path_for(ckpt_dir, rank)
    if not os.path.exists(p):
        if not reshard:
            return None
        p = _donor(ckpt_dir)
        if p is None:
            return None
        obj = torch.load(p, map_location=map_location, weights_only=True)
        if (world is None or obj.get("world") is None or int(obj["world"]) == int(world)) and (
                mode is None or obj.get("mode") in (None, mode)):
            return None  # same topology: this rank's own checkpoint is genuinely missing (agree refuses)
    else:
        obj = torch.load(p, map_location=map_location, weights_only=True)
    saved_w, saved_m = obj.get("world"), obj.get("mode")
    mismatch = []
    if world is not None and saved_w is not None and int(saved_w) != int(world):
        mismatch.append(f"world size {saved_w} -> {world}")
    if mode is not None and saved_m is not None and saved_m != mode:
        mismatch.append(f"sync mode {saved_m!r} -> {mode!r}")
    if mismatch:
        what = ", ".join(mismatch)
        if not reshard:
            raise ResumeMismatch(f"{p} was written by a different topology ({what}); its batch index refers to "
                                 f"another data shard. Pass --resume-reshard to load the weights and restart "
                                 f"the epoch at batch 0.")
        warnings.warn(f"resuming {p} across a topology change ({what}): restarting epoch {obj['epoch']} at batch 0")
        obj = dict(obj, batch_idx=0)
    engine.load_state_dict(obj["model"])
    engine.load_optimizer_state_dict(obj["optimizer"])
    if "steps_taken" in obj:
        engine.steps_taken = int(obj["steps_taken"])
    if "rng" in obj:
        torch.set_rng_state(obj["rng"])
    return obj


def _donor(ckpt_dir: str) -> Optional[str]:
    """Lowest-numbered rank file in ckpt_dir (the checkpoint a new rank of a grown world loads)."""
    if not os.path.isdir(ckpt_dir):
        return None
    ranks = sorted(int(f[4:-3]) for f in os.listdir(ckpt_dir)
                   if f.startswith("rank") and f.endswith(".pt") and f[4:-3].isdigit())
    return path_for(ckpt_dir, ranks[0]) if ranks else None


def resume_point(obj: Optional[dict]) -> Tuple[int, int, int, int]:
    """(has_checkpoint, epoch, batch_idx, steps_taken) of a loaded checkpoint (zeros if none)."""
    if obj is None:
        return 0, 0, 0, 0
    return 1, int(obj["epoch"]), int(obj["batch_idx"]), int(obj.get("steps_taken", 0))


def _pieces(point) -> list:
    """Each value (>= -1, < 2^48 - 1) as three exact 16-bit pieces of value + 1: a float32 all-reduce
    then compares them exactly (a float32 of a large step count would round)."""
    out = []
    for x in point:
        v = int(x) + 1
        if v < 0 or v >= 1 << 48:
            raise ValueError(f"resume point value out of range: {x}")
        out += [(v >> 32) & 0xFFFF, (v >> 16) & 0xFFFF, v & 0xFFFF]
    return out


def _unpieces(p) -> list:
    return [(int(p[i]) << 32 | int(p[i + 1]) << 16 | int(p[i + 2])) - 1 for i in range(0, len(p), 3)]


def agree(comm, point: Tuple[int, int, int, int], device) -> None:
    """Raise ResumeMismatch on EVERY rank unless all ranks hold the same resume point.  One max
    all-reduce of (x, -x) over exact 16-bit pieces: max(x) == -max(-x) == min(x) iff all agree."""
    if comm.world <= 1:
        return
    v = torch.tensor(_pieces(point), dtype=torch.float64)
    t = torch.cat([v, -v]).to(device=device, dtype=torch.float32 if device.type == "cuda" else torch.float64)
    with comm.region():
        comm.all_reduce(t, "max")
    comm.wait()
    t = t.double().cpu()
    k = v.numel()
    mx, mn = t[:k], -t[k:]
    if not torch.equal(mx, mn):
        raise ResumeMismatch(f"ranks disagree on the resume point (has_ckpt, epoch, batch_idx, steps_taken): "
                             f"max {_unpieces(mx.tolist())} vs min {_unpieces(mn.tolist())}, this rank "
                             f"{list(point)}; refusing to pair gradients of different steps")
