"""Per-rank checkpoint / resume (new scope: the reference has none — SURVEY §5.4).

Layout: ``<dir>/rank{R}.pt`` holding

    {"model": reference-layout state_dict (58 keys for VGG-11, OIHW fp32; "module." prefix when
               saved from DDP mode, as DistributedDataParallel.state_dict() would),
     "optimizer": torch.optim.SGD state_dict (momentum_buffer per param),
     "epoch": int, "batch_idx": int (next batch to run), "sampler_seed": int,
     "world": int, "mode": str, "rng": torch CPU RNG state}

``model`` loads straight into ``model.VGG11().load_state_dict`` (after stripping ``module.``).
Loading uses ``torch.load(weights_only=True)`` — nothing in the file is executed.
"""
from __future__ import annotations

import os
from typing import Optional

import torch


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
        "rng": torch.get_rng_state(),
    }
    p = path_for(ckpt_dir, rank)
    tmp = p + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, p)
    return p


def load(ckpt_dir: str, rank: int, engine, map_location="cpu") -> Optional[dict]:
    p = path_for(ckpt_dir, rank)
    if not os.path.exists(p):
        return None
    obj = torch.load(p, map_location=map_location, weights_only=True)
    engine.load_state_dict(obj["model"])
    engine.load_optimizer_state_dict(obj["optimizer"])
    if "rng" in obj:
        torch.set_rng_state(obj["rng"])
    return obj
