"""Communicators: the collective layer the gradient-sync strategies run on.

``RcclComm``  — the MI355X path: the native C++ communicator (csrc/runtime/rccl_comm.cpp) straight
               on RCCL over xGMI, with its own high-priority comm HIP stream.  Bootstrapped by
               exchanging an ``ncclUniqueId`` through the rendezvous store.
``TorchComm`` — ``torch.distributed`` (gloo on CPU — the test oracle; nccl=RCCL on GPU for A/B
               comparison), with a side stream on GPU so collectives overlap compute the same way.
``NullComm``  — world size 1: every collective is the identity (gather copies).

All share one ordering contract, which is what lets backward overlap communication:

    with comm.region():          # comm stream waits for work queued so far on the compute stream
        comm.all_reduce(t)       # collectives + any kernels launched here run on the comm stream
    comm.wait()                  # compute stream waits for everything issued on the comm stream

No host synchronisation happens in any of these calls on GPU.
"""
from __future__ import annotations

import contextlib
import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist

from ..utils.streams import StreamJoin


class Comm:
    rank: int = 0
    world: int = 1
    name = "base"

    @contextlib.contextmanager
    def region(self, join: bool = True):
        """Collectives issued inside run on the communicator's stream, ordered after the work
        queued so far on the current stream (``join=False``: the caller orders them itself, e.g.
        with a kernel-start signal wait issued first inside the region)."""
        yield

    def all_reduce(self, t: torch.Tensor, op: str = "sum"):
        raise NotImplementedError

    def all_reduce_here(self, t: torch.Tensor, op: str = "sum"):
        """The collective ordered on the CURRENT stream: after everything issued on it so far and
        every earlier collective, before what follows on it.  Generic form: a region + a wait;
        RcclComm issues it on the current stream itself (no comm-stream hop)."""
        with self.region():
            self.all_reduce(t, op)
        self.wait()

    def broadcast(self, t: torch.Tensor, root: int = 0):
        raise NotImplementedError

    def gather(self, send: torch.Tensor, recv: Optional[torch.Tensor], root: int = 0):
        raise NotImplementedError

    def reduce_scatter(self, send: torch.Tensor, recv: torch.Tensor, op: str = "sum"):
        raise NotImplementedError

    def all_gather(self, send: torch.Tensor, recv: torch.Tensor):
        raise NotImplementedError

    def wait(self):
        pass

    def prepare(self, tensors):
        """Collective hint (every rank, same tensors, same order): these tensors will carry
        collectives for the communicator's lifetime (the peer-memory communicator maps them)."""

    def synchronize(self):
        pass

    def barrier(self):
        pass

    def check(self):
        """Raise if the communicator reported an asynchronous error."""

    def close(self):
        pass


class NullComm(Comm):
    name = "null"

    def __init__(self):
        self.rank, self.world = 0, 1

    def all_reduce(self, t, op="sum"):
        return None

    def broadcast(self, t, root=0):
        return None

    def gather(self, send, recv, root=0):
        if recv is not None:
            recv.view(-1)[: send.numel()].copy_(send.view(-1))

    def reduce_scatter(self, send, recv, op="sum"):
        recv.copy_(send.view(-1)[: recv.numel()].view_as(recv))

    def all_gather(self, send, recv):
        recv.view(-1)[: send.numel()].copy_(send.view(-1))


_TORCH_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
              "prod": dist.ReduceOp.PRODUCT}


class TorchComm(Comm):
    """torch.distributed process group.  Every op waits on its Work right after issue: on GPU
    (nccl) that is a device-side wait of the side stream, on CPU (gloo) a host wait.

    GPU tensors over a gloo group (``--comm gloo``: several ranks sharing one GPU, which RCCL does
    not allow — the multi-rank rehearsal of the GPU engine on a one-GPU box) are staged through
    host memory: the side stream is drained, the collective runs on a CPU copy, the result is
    copied back on the side stream."""

    name = "torch"

    def __init__(self, group=None, device: Optional[torch.device] = None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.side = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self.stage = self.device.type == "cuda" and dist.get_backend(group) == "gloo"
        if self.stage:
            self.name = "gloo-staged"
        self._join_in = StreamJoin() if self.side is not None else None
        self._join_out = StreamJoin() if self.side is not None else None

    @contextlib.contextmanager
    def region(self, join: bool = True):
        if self.side is None:
            yield
            return
        if join:
            self._join_in(self.side, torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.side):
            yield

    def _w(self, work):
        if work is not None:
            work.wait()

    def _staged(self, fn, *ts):
        """Run fn on host copies of ts (gloo + GPU tensors), then copy every result back."""
        hs = [t.detach().cpu() for t in ts]  # drains the current (side) stream up to here
        fn(*hs)
        for t, h in zip(ts, hs):
            t.copy_(h)

    def all_reduce(self, t, op="sum"):
        if self.stage:
            self._staged(lambda h: dist.all_reduce(h, dist.ReduceOp.SUM if op == "avg" else _TORCH_OPS[op],
                                                   group=self.group), t)
            if op == "avg":
                t.div_(self.world)
            return
        if op == "avg":
            self._w(dist.all_reduce(t, dist.ReduceOp.SUM, group=self.group, async_op=True))
            t.div_(self.world)
            return
        self._w(dist.all_reduce(t, _TORCH_OPS[op], group=self.group, async_op=True))

    def broadcast(self, t, root=0):
        if self.stage:
            self._staged(lambda h: dist.broadcast(h, src=root, group=self.group), t)
            return
        self._w(dist.broadcast(t, src=root, group=self.group, async_op=True))

    def gather(self, send, recv, root=0):
        if self.stage:
            hs = send.detach().cpu()
            hr = recv.detach().cpu() if self.rank == root else None
            dist.gather(hs.view(-1), gather_list=list(hr.view(self.world, -1).unbind(0)) if hr is not None else None,
                        dst=root, group=self.group)
            if hr is not None:
                recv.copy_(hr)
            return
        gl = list(recv.view(self.world, -1).unbind(0)) if self.rank == root else None
        self._w(dist.gather(send.view(-1), gather_list=gl, dst=root, group=self.group, async_op=True))

    def reduce_scatter(self, send, recv, op="sum"):
        if self.device.type == "cpu" or self.stage:  # gloo has no reduce_scatter: all_reduce a copy, keep own shard
            tmp = send.clone()
            self.all_reduce(tmp, op)
            recv.copy_(tmp.view(self.world, -1)[self.rank].view_as(recv))
            return
        self._w(dist.reduce_scatter_tensor(recv, send, _TORCH_OPS[op], group=self.group, async_op=True))

    def all_gather(self, send, recv):
        if self.stage:
            hs, hr = send.detach().cpu(), recv.detach().cpu()
            dist.all_gather(list(hr.view(self.world, -1).unbind(0)), hs.view(-1), group=self.group)
            recv.copy_(hr)
            return
        if self.device.type == "cpu":  # gloo: list form (send may alias its slot of recv)
            src = send.clone()
            self._w(dist.all_gather(list(recv.view(self.world, -1).unbind(0)), src.view(-1), group=self.group,
                                    async_op=True))
            return
        self._w(dist.all_gather_into_tensor(recv, send, group=self.group, async_op=True))

    def wait(self):
        if self.side is not None:
            self._join_out(torch.cuda.current_stream(self.device), self.side)

    def synchronize(self):
        if self.side is not None:
            self.side.synchronize()

    def barrier(self):
        dist.barrier(group=self.group)


def exchange_unique_id(store, rank: int, make_uid, tag: str = "dpa_rccl_uid", timeout_s: Optional[int] = None) -> bytes:
    """Rank 0 creates the RCCL unique id and publishes it in the rendezvous store; every other rank
    blocks (bounded) until it appears.  (Replaces the store half of NCCL's bootstrap.)"""
    timeout_s = timeout_s or int(os.environ.get("DPA_RCCL_INIT_TIMEOUT", "600"))
    if rank == 0:
        uid = bytes(make_uid())
        store.set(tag, uid)
        return uid
    store.wait([tag], datetime.timedelta(seconds=timeout_s))
    return bytes(store.get(tag))


class RcclComm(Comm):
    """Native RCCL communicator (one per process/GPU).

    Failure handling (native watchdog thread, csrc/runtime/rccl_comm.cpp): env
    ``DPA_COMM_TIMEOUT`` (s, default 600) bounds how long any collective may stay outstanding;
    async RCCL errors and timeouts abort the communicator and, unless ``DPA_WATCHDOG_EXIT=0``,
    end the process with exit code 70 so the launcher tears the job down.  ``DPA_DEBUG_SYNC=1``
    makes every collective host-synchronous and error-checked (ordering/race debugging).
    ``DPA_WATCHDOG=0`` disables the thread.  ``channels`` (default ``DPA_RCCL_CHANNELS``, 0 = RCCL's
    choice) bounds the workgroups the collectives run on (``ncclConfig_t.maxCTAs``): the CU
    footprint of the communication beside the overlapped backward."""

    name = "rccl"

    def __init__(self, rank: int, world: int, device: torch.device, store=None, uid: Optional[bytes] = None,
                 tag: str = "dpa_rccl_uid", channels: Optional[int] = None):
        from .. import _ext

        C = _ext.require()
        self.rank, self.world = rank, world
        self.device = torch.device(device)
        if uid is None:
            if store is None:
                raise ValueError("RcclComm needs a store (or an explicit unique id) for bootstrap")
            uid = exchange_unique_id(store, rank, C.rccl_unique_id, tag)
        with torch.cuda.device(self.device):
            self._c = C.RcclComm(rank, world, bytes(uid), self.device.index or 0,
                                 high_priority=False,
                                 timeout_s=float(os.environ.get("DPA_COMM_TIMEOUT", "600")),
                                 watchdog=os.environ.get("DPA_WATCHDOG", "1") == "1",
                                 exit_on_error=os.environ.get("DPA_WATCHDOG_EXIT", "1") == "1",
                                 debug_sync=os.environ.get("DPA_DEBUG_SYNC", "0") == "1",
                                 max_ctas=channels if channels is not None else
                                 int(os.environ.get("DPA_RCCL_CHANNELS", "0")))
        self.channels = self._c.max_ctas
        self.stream = torch.cuda.ExternalStream(self._c.stream_ptr(), device=self.device)
        self._join_in, self._join_out = StreamJoin(), StreamJoin()
        self._store = store

    @contextlib.contextmanager
    def region(self, join: bool = True):
        if join:
            self._join_in(self.stream, torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            yield

    def all_reduce(self, t, op="sum"):
        self._c.all_reduce(t, op)

    def all_reduce_here(self, t, op="sum"):
        self.wait()  # every earlier collective of this communicator first (one hop: comm -> current)
        self._c.all_reduce_here(t, op)

    def broadcast(self, t, root=0):
        self._c.broadcast(t, root)

    def gather(self, send, recv, root=0):
        self._c.gather(send, recv, root)

    def reduce_scatter(self, send, recv, op="sum"):
        self._c.reduce_scatter(send, recv, op)

    def all_gather(self, send, recv):
        self._c.all_gather(send, recv)

    def wait(self):
        self._join_out(torch.cuda.current_stream(self.device), self.stream)

    def synchronize(self):
        self._c.synchronize()

    def barrier(self):
        t = torch.zeros(1, device=self.device)
        with self.region():
            self.all_reduce(t)
        self.wait()
        torch.cuda.current_stream(self.device).synchronize()

    def check(self):
        err = self._c.async_error()
        if err:
            raise RuntimeError(f"RCCL async error on rank {self.rank}: {err}")

    def close(self):
        try:
            self._c.synchronize()
        except Exception:
            self._c.abort()

    def abort(self):
        self._c.abort()

    def outstanding(self) -> int:
        """Collectives issued whose completion the watchdog has not yet observed."""
        return self._c.outstanding()

    def ops_issued(self) -> int:
        return self._c.ops_issued()

    def comm_count(self) -> int:
        """Ranks in the communicator as RCCL reports them (ncclCommCount); -1 once aborted."""
        return self._c.comm_count()
