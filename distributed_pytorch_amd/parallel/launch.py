"""Process-group bootstrap for both of the reference's launch styles.

* CLI style (main_gather.py:97-107, main_all_reduce.py:86-96, main_part3.py:78-88):
  ``--master-ip IP --num-nodes N --rank R`` → rendezvous at ``tcp://IP:6585``.
* torchrun style (main_ddp.py:93-104, start_ddp.sh): MASTER_ADDR/MASTER_PORT/WORLD_SIZE/RANK/
  LOCAL_RANK from the environment (``env://``).

One process per GPU: LOCAL_RANK (or rank mod #GPUs) selects the device.  Rendezvous
(``DPA_RENDEZVOUS``):
* ``native`` (default on GPU): no torch.distributed at all — the native C++ TCP store
  (parallel/store.py, csrc/runtime/tcp_store.cpp) on MASTER_ADDR:DPA_STORE_PORT bootstraps RCCL
  (ncclUniqueId exchange) and provides the CPU-side barriers;
* ``torch`` (default on CPU, and for ``--comm torch``): a torch.distributed gloo group carries the
  rendezvous store and barriers — on CPU it is also the communicator (the multi-process test oracle).
On GPU the gradient collectives go through the native RCCL communicator (``comm="rccl"``), the
peer-memory kernels alone (``comm="ipc"``, one node: HIP IPC mappings, several ranks may share a
GPU; parallel/ipc.py), or torch's own nccl group (``comm="torch"``, torch rendezvous only) for A/B
comparison.
There is no silent fallback: if the native communicator cannot be created the job fails
(``DPA_COMM_FALLBACK=1`` opts into torch's nccl group instead, which the bench reports).
"""
from __future__ import annotations

import datetime
import os
import time
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from .comm import Comm, NullComm, RcclComm, TorchComm
from .store import NativeStore

DEFAULT_PORT = 6585  # main_gather.py:107


@dataclass
class DistContext:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    comm: Comm
    initialized_pg: bool
    store: Optional[NativeStore] = None
    _nbar: int = 0

    def barrier(self):
        """CPU-side barrier over all ranks (gloo group or native store)."""
        if self.initialized_pg:
            dist.barrier()
        elif self.store is not None:
            self._nbar += 1
            self.store.barrier(f"ctx_barrier_{self._nbar}")

    def all_max(self, value: float) -> float:
        if self.initialized_pg:
            t = torch.tensor([float(value)], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t[0])
        if self.store is not None:
            self._nbar += 1
            return self.store.all_max(f"ctx_max_{self._nbar}", value)
        return float(value)

    def shutdown(self):
        try:
            self.comm.close()
        finally:
            if self.initialized_pg and dist.is_initialized():
                dist.destroy_process_group()
            if self.store is not None:
                self.store.close()


def _timeout():
    return datetime.timedelta(seconds=int(os.environ.get("DPA_PG_TIMEOUT", "1800")))


def pick_device(local_rank: int, want: str = "auto") -> torch.device:
    # RCCL and CUDA-tensor sharing across processes need the dmabuf IPC path on this platform
    # (legacy IPC fails with hipIpcGetMemHandle: invalid argument).  spawn.py sets it for its ranks;
    # under torchrun or a hand launch it must be in the environment before the HIP runtime starts,
    # i.e. before the first torch.cuda query below.
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if want == "cpu" or (want == "auto" and not torch.cuda.is_available()):
        return torch.device("cpu")
    n = torch.cuda.device_count()
    if n == 0:
        raise RuntimeError("GPU requested but none visible")
    d = torch.device("cuda", local_rank % n)
    torch.cuda.set_device(d)
    return d


def _rendezvous(device: torch.device, comm: str = "rccl") -> str:
    r = os.environ.get("DPA_RENDEZVOUS", "auto")
    if r not in ("auto", "torch", "native"):
        raise ValueError("DPA_RENDEZVOUS must be 'auto', 'torch' or 'native'")
    if r == "auto":
        return "native" if device.type == "cuda" and comm in ("rccl", "ipc") else "torch"
    return r


def _native_store(host: str, port: int, rank: int, world: int) -> NativeStore:
    return NativeStore(host, port, rank, world, timeout_s=_timeout().total_seconds())


def native_store_from_env(rank: int, world: int) -> NativeStore:
    """The native rendezvous store of an env:// job.  Its port:
    * ``DPA_STORE_PORT`` when set (the framework's own launcher picks a free one);
    * under torchrun (``TORCHELASTIC_USE_AGENT_STORE=True``): rank 0 binds an ephemeral port and
      publishes it through the elastic agent's store at MASTER_PORT — one key, read by the other
      ranks; no process group is created — so a busy neighbouring port cannot break the job;
    * otherwise MASTER_PORT + 1."""
    host = os.environ["MASTER_ADDR"]
    if "DPA_STORE_PORT" in os.environ:
        return _native_store(host, int(os.environ["DPA_STORE_PORT"]), rank, world)
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":
        agent = dist.TCPStore(host, int(os.environ["MASTER_PORT"]), None, False, _timeout())
        key = "dpa/native_store_port/{}/{}".format(os.environ.get("TORCHELASTIC_RUN_ID", "run"),
                                                   os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
        if rank == 0:
            st = _native_store(host, 0, rank, world)
            agent.set(key, str(st.port))
            return st
        return _native_store(host, int(agent.get(key).decode()), rank, world)
    return _native_store(host, int(os.environ["MASTER_PORT"]) + 1, rank, world)


def _make_comm(kind: str, rank: int, world: int, device: torch.device, store=None) -> Comm:
    if world == 1:
        # DPA_FORCE_COMM=1 runs the real RCCL communicator even on one GPU (a 1-rank communicator:
        # every collective is an identity), exercising the stream/event/bucket path on a 1-GPU box
        if os.environ.get("DPA_FORCE_COMM", "0") == "1" and device.type == "cuda":
            from .. import _ext

            return RcclComm(0, 1, device, uid=_ext.require().rccl_unique_id())
        return NullComm()
    if device.type != "cuda":
        if store is not None:
            raise RuntimeError("native rendezvous drives RCCL only: use DPA_RENDEZVOUS=torch (gloo) on CPU")
        return TorchComm(device=device)
    if kind == "ipc":  # peer-memory collectives only (parallel/ipc.py): no host staging, no RCCL
        from .ipc import IpcComm

        if store is None:
            store = dist.distributed_c10d._get_default_store()
        return IpcComm(None, store, device, rank=rank, world=world)
    if kind == "gloo":  # GPU tensors staged through gloo: several ranks may share one GPU (rehearsal)
        if store is not None:
            raise RuntimeError("--comm gloo needs the torch rendezvous")
        return TorchComm(device=device)
    if kind == "torch":
        if store is not None:
            raise RuntimeError("--comm torch needs the torch rendezvous")
        group = dist.new_group(backend="nccl")
        return TorchComm(group=group, device=device)
    torch_store = store is None
    if torch_store:
        store = dist.distributed_c10d._get_default_store()
    try:
        t0 = time.perf_counter()
        comm = RcclComm(rank, world, device, store=store)
        comm.init_s = time.perf_counter() - t0  # (reported by bench.py: first-contact diagnostics)
    except Exception as e:  # noqa: BLE001 — keep the job alive on torch's own RCCL group
        if not torch_store or os.environ.get("DPA_COMM_FALLBACK", "0") != "1":
            raise
        print(f"[rank {rank}] native RCCL communicator failed ({e}); falling back to torch's nccl (RCCL) group",
              flush=True)
        return TorchComm(group=dist.new_group(backend="nccl"), device=device)
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
    init, store = False, None
    if num_nodes > 1:
        if _rendezvous(dev, comm) == "native":
            store = _native_store(master_ip, port, rank, num_nodes)
        else:
            dist.init_process_group(backend="gloo", init_method=f"tcp://{master_ip}:{port}", world_size=num_nodes,
                                    rank=rank, timeout=_timeout())
            init = True
    return DistContext(rank, num_nodes, local_rank, dev, _make_comm(comm, rank, num_nodes, dev, store), init, store)


def env_dict():
    keys = ("MASTER_ADDR", "MASTER_PORT", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "LOCAL_RANK", "RANK")
    return {k: os.environ[k] for k in keys}


def init_env(device: str = "auto", comm: str = "rccl") -> DistContext:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = pick_device(local_rank, device)
    init, store = False, None
    if world > 1:
        if _rendezvous(dev, comm) == "native":
            store = native_store_from_env(rank, world)
        else:
            dist.init_process_group(backend="gloo", init_method="env://", timeout=_timeout())
            init = True
    return DistContext(rank, world, local_rank, dev, _make_comm(comm, rank, world, dev, store), init, store)


def init_single(device: str = "auto") -> DistContext:
    dev = pick_device(0, device)
    return DistContext(0, 1, 0, dev, NullComm(), False)
