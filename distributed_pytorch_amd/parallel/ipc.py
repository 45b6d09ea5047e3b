"""Peer-memory all-reduce: ``IpcComm`` routes SUM all-reduces of registered GPU memory through the
native two-shot peer kernel (csrc/kernels/ipc_allreduce.hip, csrc/runtime/ipc_comm.cpp) and every
other collective through the communicator it wraps (RCCL, or gloo when several ranks share one GPU).

Why: the reference's whole purpose is the gradient exchange (main_all_reduce.py:45-48,
main_ddp.py:137).  On an 8-GPU MI355X node every rank can map its peers' gradient arenas over xGMI
and reduce them with one kernel on a fixed workgroup budget; and on a one-GPU lease,
where RCCL refuses two ranks on one device, the same kernel is the only device-side multi-rank
collective that can run at all (ranks sharing the GPU map each other's memory through HIP IPC).

Bootstrap: every rank publishes the handles of its signal array and staging buffer through the
rendezvous store and opens its peers'; memory the peer kernel may reduce (the gradient arena) is
registered explicitly (``register``, collective, every rank in the same order) the same way.
Creation runs a self-check all-reduce with exact integer sums; a failed or timed-out check raises.
Results are bitwise identical on every rank (each element summed once, in rank order).
"""
from __future__ import annotations

import contextlib
import datetime
import os
from typing import Dict, Optional, Tuple

import torch

from .comm import Comm


def _store_exchange(store, tag: str, rank: int, world: int, value: bytes, timeout_s: float) -> list:
    store.set(f"{tag}/{rank}", value)
    keys = [f"{tag}/{w}" for w in range(world)]
    store.wait(keys, datetime.timedelta(seconds=timeout_s))
    return [bytes(store.get(k)) for k in keys]


class IpcComm(Comm):
    """``inner``: the communicator for everything but SUM all-reduces of 16-byte aligned fp32 GPU
    tensors (its stream is the comm stream of both).  ``store``: rendezvous store shared by the ranks
    (NativeStore or a torch store).  ``blocks``: workgroups per rank (DPA_IPC_BLOCKS, default 32)."""

    name = "ipc"

    def __init__(self, inner: Comm, store, device: torch.device, blocks: Optional[int] = None,
                 stage_floats: int = 1 << 22, timeout_s: Optional[float] = None, tag: str = "dpa_ipc"):
        from .. import _ext

        C = _ext.require()
        self.inner = inner
        self.rank, self.world = inner.rank, inner.world
        self.device = torch.device(device)
        self.store = store
        self.tag = tag
        self.blocks = int(blocks or os.environ.get("DPA_IPC_BLOCKS", "32"))
        self.timeout_s = float(timeout_s if timeout_s is not None else os.environ.get("DPA_IPC_TIMEOUT", "60"))
        # elements one collective can carry: each rank stages a 1/W slice (multiple of 4 elements)
        self.max_elems = (int(stage_floats) // 4 * 4) * self.world
        self._nreg = 0
        self._regions: Dict[Tuple[int, int], int] = {}  # (data ptr, elements) -> region id
        with torch.cuda.device(self.device):
            self._c = C.IpcComm(self.rank, self.world, self.device.index or 0, int(stage_floats))
        sig = _store_exchange(store, f"{tag}/sig", self.rank, self.world, bytes(self._c.sig_handle()), 600.0)
        stg = _store_exchange(store, f"{tag}/stage", self.rank, self.world, bytes(self._c.stage_handle()), 600.0)
        with torch.cuda.device(self.device):
            self._c.set_peers(sig, stg)
        self.ipc_ops = 0
        self._self_check()

    # ---- Comm interface ----
    @property
    def stream(self):
        return getattr(self.inner, "stream", None) or getattr(self.inner, "side", None)

    @contextlib.contextmanager
    def region(self, join: bool = True):
        with self.inner.region(join):
            yield

    def register(self, t: torch.Tensor) -> None:
        """Collective (every rank, same order): make t's memory reachable by the peer kernel.  Only
        registered memory goes through it -- a registration pins the peers' mappings of that memory,
        so it must outlive the communicator (the gradient arena does)."""
        from .. import _ext

        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            raise ValueError("IpcComm.register: contiguous fp32 GPU tensor expected")
        hs = _store_exchange(self.store, f"{self.tag}/reg{self._nreg}", self.rank, self.world,
                             bytes(_ext.require().IpcComm.tensor_handle(t)), 600.0)
        self._nreg += 1
        with torch.cuda.device(self.device):
            rid = self._c.add_region(hs, t)
        self._regions[(t.data_ptr(), t.numel())] = rid
        self._keep = getattr(self, "_keep", []) + [t]

    def _region_of(self, t: torch.Tensor) -> Optional[Tuple[int, int]]:
        """(region id, element offset) of the registered region holding t, or None."""
        p, n = t.data_ptr(), t.numel()
        for (b, m), rid in self._regions.items():
            if b <= p and p + 4 * n <= b + 4 * m:
                return rid, (p - b) // 4
        return None

    def ipc_eligible(self, t: torch.Tensor, op: str) -> bool:
        return (op == "sum" and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
                and t.data_ptr() % 16 == 0 and self._region_of(t) is not None)

    def _peer_all_reduce(self, t: torch.Tensor):
        """One peer-kernel collective per staging-buffer-sized piece (pieces are multiples of 4*W
        elements, so every piece stays 16-byte aligned)."""
        rid, off = self._region_of(t)
        n, done = t.numel(), 0
        while done < n:
            k = min(self.max_elems, n - done)
            self._c.all_reduce(rid, off + done, k, self.blocks, int(self.timeout_s * 1e6))
            self.ipc_ops += 1
            done += k

    def all_reduce(self, t: torch.Tensor, op: str = "sum"):
        if not self.ipc_eligible(t, op):
            return self.inner.all_reduce(t, op)
        self._peer_all_reduce(t)

    def all_reduce_here(self, t: torch.Tensor, op: str = "sum"):
        if not self.ipc_eligible(t, op):
            return self.inner.all_reduce_here(t, op)
        self.inner.wait()  # earlier collectives (RCCL or peer kernels on the comm stream) first
        self._peer_all_reduce(t)

    def broadcast(self, t, root=0):
        self.inner.broadcast(t, root)

    def gather(self, send, recv, root=0):
        self.inner.gather(send, recv, root)

    def reduce_scatter(self, send, recv, op="sum"):
        self.inner.reduce_scatter(send, recv, op)

    def all_gather(self, send, recv):
        self.inner.all_gather(send, recv)

    def wait(self):
        self.inner.wait()

    def synchronize(self):
        self.inner.synchronize()

    def barrier(self):
        self.inner.barrier()

    def check(self):
        if self._c.take_timeout():
            raise RuntimeError(f"IPC all-reduce on rank {self.rank}: a peer wait timed out (results invalid)")
        self.inner.check()

    def close(self):
        self.inner.close()

    # ---- bootstrap check ----
    def _self_check(self):
        """Exact-integer all-reduce through the peer kernel (sum of rank + 1 and of a ramp), with an
        odd length that exercises the slice tails; raises unless every element is exact."""
        n = 4099
        t = torch.arange(n + 1, dtype=torch.float32, device=self.device)[:n] + float(self.rank + 1)
        self.register(t)
        with self.region():
            self.all_reduce(t)
        self.wait()
        torch.cuda.synchronize(self.device)
        if self._c.take_timeout():
            raise RuntimeError(f"IPC self-check timed out on rank {self.rank}")
        W = self.world
        exp = torch.arange(n, dtype=torch.float32) * W + W * (W + 1) / 2
        if not torch.equal(t.cpu(), exp):
            raise RuntimeError(f"IPC self-check failed on rank {self.rank}")
