"""Process-group bootstrap for both of the reference's launch styles.

* CLI style (main_gather.py:97-107, main_all_reduce.py:86-96, main_part3.py:78-88):
  ``--master-ip IP --num-nodes N --rank R`` → rendezvous at ``tcp://IP:6585``.
* torchrun style (main_ddp.py:93-104, start_ddp.sh): MASTER_ADDR/MASTER_PORT/WORLD_SIZE/RANK/
  LOCAL_RANK from the environment (``env://``).

One process per GPU: LOCAL_RANK (or rank mod #GPUs) selects the device.  The torch.distributed
process group (gloo) carries the rendezvous store and CPU-side barriers; on GPU the gradient
collectives go through the native RCCL communicator bootstrapped from that store (``comm="rccl"``),
or through torch's own nccl group (``comm="torch"``) for A/B comparison.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from .comm import Comm, NullComm, RcclComm, TorchComm

DEFAULT_PORT = 6585  # main_gather.py:107


@dataclass
class DistContext:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    comm: Comm
    initialized_pg: bool

    def shutdown(self):
        try:
            self.comm.close()
        finally:
            if self.initialized_pg and dist.is_initialized():
                dist.destroy_process_group()


def _timeout():
    return datetime.timedelta(seconds=int(os.environ.get("DPA_PG_TIMEOUT", "1800")))


def pick_device(local_rank: int, want: str = "auto") -> torch.device:
    if want == "cpu" or (want == "auto" and not torch.cuda.is_available()):
        return torch.device("cpu")
    n = torch.cuda.device_count()
    if n == 0:
        raise RuntimeError("GPU requested but none visible")
    d = torch.device("cuda", local_rank % n)
    torch.cuda.set_device(d)
    return d


def _make_comm(kind: str, rank: int, world: int, device: torch.device) -> Comm:
    if world == 1:
        # DPA_FORCE_COMM=1 runs the real RCCL communicator even on one GPU (a 1-rank communicator:
        # every collective is an identity), exercising the stream/event/bucket path on a 1-GPU box
        if os.environ.get("DPA_FORCE_COMM", "0") == "1" and device.type == "cuda":
            from .. import _ext

            return RcclComm(0, 1, device, uid=_ext.require().rccl_unique_id())
        return NullComm()
    if device.type != "cuda":
        return TorchComm(device=device)
    if kind == "torch":
        group = dist.new_group(backend="nccl")
        return TorchComm(group=group, device=device)
    store = dist.distributed_c10d._get_default_store()
    comm = RcclComm(rank, world, device, store=store)
    # correctness-by-construction check of the fresh communicator: sum of (rank+1)
    t = torch.full((8,), float(rank + 1), device=device)
    with comm.region():
        comm.all_reduce(t)
    comm.wait()
    exp = world * (world + 1) / 2
    if not torch.allclose(t.cpu(), torch.full((8,), exp)):
        raise RuntimeError(f"RCCL self-check failed on rank {rank}: got {t.cpu().tolist()}, expected {exp}")
    return comm


def init_cli(master_ip: str, num_nodes: int, rank: int, port: int = DEFAULT_PORT, device: str = "auto",
             comm: str = "rccl") -> DistContext:
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    dev = pick_device(local_rank, device)
    init = False
    if num_nodes > 1:
        dist.init_process_group(backend="gloo", init_method=f"tcp://{master_ip}:{port}", world_size=num_nodes,
                                rank=rank, timeout=_timeout())
        init = True
    return DistContext(rank, num_nodes, local_rank, dev, _make_comm(comm, rank, num_nodes, dev), init)


def env_dict():
    keys = ("MASTER_ADDR", "MASTER_PORT", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "LOCAL_RANK", "RANK")
    return {k: os.environ[k] for k in keys}


def init_env(device: str = "auto", comm: str = "rccl") -> DistContext:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = pick_device(local_rank, device)
    init = False
    if world > 1:
        dist.init_process_group(backend="gloo", init_method="env://", timeout=_timeout())
        init = True
    return DistContext(rank, world, local_rank, dev, _make_comm(comm, rank, world, dev), init)


def init_single(device: str = "auto") -> DistContext:
    dev = pick_device(0, device)
    return DistContext(0, 1, 0, dev, NullComm(), False)
