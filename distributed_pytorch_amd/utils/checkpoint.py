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
  weights and optimizer state anyway and restarts the saved epoch at batch 0;
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
        return None
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


def resume_point(obj: Optional[dict]) -> Tuple[int, int, int, int]:
    """(has_checkpoint, epoch, batch_idx, steps_taken) of a loaded checkpoint (zeros if none)."""
    if obj is None:
        return 0, 0, 0, 0
    return 1, int(obj["epoch"]), int(obj["batch_idx"]), int(obj.get("steps_taken", 0))


def agree(comm, point: Tuple[int, int, int, int], device) -> None:
    """Raise ResumeMismatch on EVERY rank unless all ranks hold the same resume point.  One
    all-reduce of (x, -x): max(x) == -max(-x) == min(x) iff all ranks agree."""
    if comm.world <= 1:
        return
    v = torch.tensor(list(point), dtype=torch.float64)
    t = torch.cat([v, -v]).to(device=device, dtype=torch.float32 if device.type == "cuda" else torch.float64)
    with comm.region():
        comm.all_reduce(t, "max")
    comm.wait()
    t = t.double().cpu()
    mx, mn = t[:4], -t[4:]
    if not torch.equal(mx, mn):
        raise ResumeMismatch(f"ranks disagree on the resume point (has_ckpt, epoch, batch_idx, steps_taken): "
                             f"max {mx.long().tolist()} vs min {mn.long().tolist()}, this rank "
                             f"{list(point)}; refusing to pair gradients of different steps")
