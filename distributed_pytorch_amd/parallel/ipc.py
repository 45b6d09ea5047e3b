"""Peer-memory communicator: every collective the four sync modes use -- all-reduce (sum / max /
min), broadcast, gather, reduce-scatter, all-gather and a device barrier -- as one native kernel
per collective over HIP IPC mappings of the peers' memory (csrc/kernels/ipc_coll.hip,
csrc/runtime/ipc_comm.cpp).

Why: the reference's whole purpose is the gradient exchange (main_gather.py:49,59,
main_all_reduce.py:45-48, main_ddp.py:137).  On an 8-GPU MI355X node every rank maps its peers'
arenas over xGMI and moves them with one kernel on a fixed workgroup budget; on a
one-GPU lease, where RCCL refuses two ranks on one device, the same kernels are the only device-side
multi-rank path that can run at all (ranks sharing the GPU map each other's memory through HIP IPC).

Two ways to use it:
* standalone (``inner=None``, ``--comm ipc``): the communicator of the job.  It owns its comm
  stream; no tensor byte goes through the host, gloo or RCCL (``inner_tensor_ops`` stays 0);
* wrapping another communicator (``bench.py --ipc on|auto`` over RCCL): the collectives it can run
  go through the peer kernel, anything else (non-fp32 reductions) through ``inner``.

Memory: ``register`` (collective: every rank, same tensors, same order) makes a tensor's memory
readable by the peers in place; the sync strategies register the engine's arenas through
``prepare``.  Any other device tensor is "bounced": the kernel first copies it into this rank's
inbox (pieces of at most ``inbox_words`` words).  A registered input must sit at the same word
offset of its region on every rank (true of the arenas: same model, same layout), except in the
in-place all-gather, where each rank's input is its own slot of the output (ZeRO-1's form).

Bootstrap: every rank publishes the handles of its signal array, staging buffer and inbox through
the rendezvous store (keys namespaced per communicator instance) and opens its peers'.  A rank that
fails during bootstrap raises a shared failure key, so its peers stop waiting and raise too instead
of blocking on the store.  Creation ends with a self-check (exact integer sums through the
registered and the bounced path) whose verdict is agreed through the store: either every rank
raises or none does.  Results are bitwise identical on every rank (each element reduced once, in
rank order).  Collectives must not be captured in a HIP graph (the signal epochs are launch
arguments; a replay would reuse them) -- they raise if the stream is capturing.
"""
from __future__ import annotations

import contextlib
import datetime
import json
import os
import time
from collections import Counter
from typing import List, Optional, Tuple

import torch

from ..utils.streams import StreamJoin
from .comm import Comm

_RED = {"sum": 0, "max": 1, "min": 2}


class IpcComm(Comm):
    """``inner``: communicator for what the peer kernel does not run (None: standalone; then
    ``rank``/``world`` are required).  ``store``: rendezvous store shared by the ranks (NativeStore
    or a torch store).  ``blocks``: workgroups per rank (DPA_IPC_BLOCKS, default 32)."""

    name = "ipc"
    _instances = 0  # every rank creates its communicators in the same order: same tag everywhere

    def __init__(self, inner: Optional[Comm], store, device: torch.device, blocks: Optional[int] = None,
                 stage_words: int = 1 << 22, inbox_words: int = 1 << 22, timeout_s: Optional[float] = None,
                 tag: str = "dpa_ipc", rank: Optional[int] = None, world: Optional[int] = None):
        from .. import _ext

        C = _ext.require()
        self.inner = inner
        if inner is not None:
            self.rank, self.world = inner.rank, inner.world
        else:
            if rank is None or world is None:
                raise ValueError("standalone IpcComm needs rank and world")
            self.rank, self.world = int(rank), int(world)
        if self.inner is None:
            self.name = "ipc-standalone"
        self.device = torch.device(device)
        self.store = store
        self.tag = f"{tag}/{IpcComm._instances}"
        IpcComm._instances += 1
        self.blocks = int(blocks or os.environ.get("DPA_IPC_BLOCKS", "32"))
        self.timeout_s = float(timeout_s if timeout_s is not None else os.environ.get("DPA_IPC_TIMEOUT", "60"))
        self.boot_timeout_s = float(os.environ.get("DPA_IPC_BOOT_TIMEOUT", "120"))
        self._tmo_us = int(self.timeout_s * 1e6)
        self._nreg = 0
        self._verify = os.environ.get("DPA_IPC_VERIFY", "0") == "1"
        self._regions: List[Tuple[int, int, int]] = []  # (data ptr, bytes, region id)
        self._keep: List[torch.Tensor] = []
        self.ops: Counter = Counter()
        self.inner_tensor_ops = 0  # collectives handed to the wrapped communicator after creation
        self.side = None
        if self.inner is None and self.device.type == "cuda":
            self.side = torch.cuda.Stream(self.device)
            self._join_in, self._join_out = StreamJoin(), StreamJoin()
        try:
            with torch.cuda.device(self.device):
                self._c = C.IpcComm(self.rank, self.world, self.device.index or 0, int(stage_words), int(inbox_words))
            sig = self._exchange("sig", bytes(self._c.sig_handle()))
            stg = self._exchange("stage", bytes(self._c.stage_handle()))
            box = self._exchange("inbox", bytes(self._c.inbox_handle()))
            with torch.cuda.device(self.device):
                self._c.set_peers(sig, stg, box)
            ok = self._self_check()
        except Exception:
            self._fail()
            raise
        if not self.agree(ok):
            raise RuntimeError(f"IPC self-check failed or timed out on some rank (rank {self.rank}: ok={ok})")
        self.ops.clear()

    # ---- store helpers (bootstrap) ----
    def _fail(self):
        try:
            self.store.add(f"{self.tag}/fail", 1)
        except Exception:  # noqa: BLE001 -- the store itself may be what failed
            pass

    def _wait(self, keys: List[str]):
        deadline = time.monotonic() + self.boot_timeout_s
        while True:
            try:
                self.store.wait(keys, datetime.timedelta(seconds=1.0))
                return
            except Exception:  # noqa: BLE001 -- one slice of the bounded wait ran out
                if self.store.add(f"{self.tag}/fail", 0) > 0:
                    raise RuntimeError(f"IpcComm rank {self.rank}: a peer failed during bootstrap") from None
                if time.monotonic() > deadline:
                    raise

    def _exchange(self, name: str, value: bytes) -> List[bytes]:
        self.store.set(f"{self.tag}/{name}/{self.rank}", value)
        keys = [f"{self.tag}/{name}/{w}" for w in range(self.world)]
        self._wait(keys)
        return [bytes(self.store.get(k)) for k in keys]

    def agree(self, ok: bool) -> bool:
        """True on every rank iff ``ok`` on every rank (host-side, through the store)."""
        self._nreg += 1
        vals = self._exchange(f"agree{self._nreg}", b"1" if ok else b"0")
        return all(v == b"1" for v in vals)

    # ---- memory ----
    def register(self, t: torch.Tensor) -> None:
        """Collective (every rank, same order): make t's memory readable by the peer kernels in
        place.  A registration pins the peers' mappings of that memory, so it must outlive the
        communicator (the engine's arenas do).  Memory already inside a registered region is not
        registered again."""
        from .. import _ext

        if not (t.is_cuda and t.is_contiguous() and t.numel() > 0 and (t.numel() * t.element_size()) % 4 == 0):
            raise ValueError("IpcComm.register: contiguous GPU tensor of whole 4-byte words expected")
        if self._loc(t)[0] >= 0:
            return
        self._nreg += 1
        hs = self._exchange(f"reg{self._nreg}", bytes(_ext.require().IpcComm.tensor_handle(t)))
        with torch.cuda.device(self.device):
            rid = self._c.add_region(hs, t)
        self._regions.append((t.data_ptr(), t.numel() * t.element_size(), rid))
        self._keep.append(t)

    def prepare(self, tensors) -> None:
        for t in tensors:
            if t is not None and t.is_cuda and t.numel() > 0:
                self.register(t)

    def _loc(self, t: torch.Tensor, kind: str = "") -> Tuple[int, int]:
        """(region id, word offset) of the registered region holding t, or (-1, 0): bounced.

        A registered collective reads every peer's copy at the SAME (region, offset); nothing in
        the kernel can tell if a peer resolved its tensor differently.  ``DPA_IPC_VERIFY=1`` (tests,
        debugging) agrees (kind, region, offset) across the ranks through the store before every
        collective and raises on a mismatch (a host round trip per collective: debug only)."""
        p, nb = t.data_ptr(), t.numel() * t.element_size()
        loc = (-1, 0)
        for b, m, rid in self._regions:
            if b <= p and p + nb <= b + m and (p - b) % 4 == 0:
                loc = (rid, (p - b) // 4)
                break
        if self._verify and kind:
            self._nreg += 1
            mine = f"{kind}:{loc[0]}:{loc[1] if loc[0] >= 0 else 0}".encode()
            vals = self._exchange(f"loc{self._nreg}", mine)
            if any(v != mine for v in vals):
                raise RuntimeError(f"IpcComm rank {self.rank}: ranks resolved the {kind} input differently "
                                   f"({[v.decode() for v in vals]}); a registered collective would read the "
                                   "wrong peer memory")
        return loc

    def _words_ok(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.is_contiguous() and (t.numel() * t.element_size()) % 4 == 0
                and t.data_ptr() % 4 == 0)

    def _guard(self):
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("IpcComm collectives cannot be captured in a HIP graph (per-launch signal epochs)")

    def _inner(self, what: str):
        if self.inner is None:
            raise ValueError(f"IpcComm (standalone): {what} is not supported by the peer kernels")
        self.inner_tensor_ops += 1
        return self.inner

    # ---- Comm interface ----
    @property
    def stream(self):
        if self.inner is None:
            return self.side
        return getattr(self.inner, "stream", None) or getattr(self.inner, "side", None)

    @contextlib.contextmanager
    def region(self, join: bool = True):
        if self.inner is not None:
            with self.inner.region(join):
                yield
            return
        if join:
            self._join_in(self.side, torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.side):
            yield

    def wait(self):
        if self.inner is not None:
            self.inner.wait()
        else:
            self._join_out(torch.cuda.current_stream(self.device), self.side)

    def ipc_eligible(self, t: torch.Tensor, op: str) -> bool:
        return self._words_ok(t) and t.dtype == torch.float32 and op in _RED

    def all_reduce(self, t: torch.Tensor, op: str = "sum"):
        o = "sum" if op == "avg" else op
        if not self.ipc_eligible(t, o):
            return self._inner(f"all_reduce({op}, {t.dtype})").all_reduce(t, op)
        self._guard()
        rid, off = self._loc(t, "all_reduce")
        self._c.all_reduce(rid, off, t, _RED[o], self.blocks, self._tmo_us)
        self.ops["all_reduce" if rid >= 0 else "all_reduce_bounced"] += 1
        if op == "avg":
            t.div_(self.world)

    def all_reduce_here(self, t: torch.Tensor, op: str = "sum"):
        if not self.ipc_eligible(t, op):
            return self._inner(f"all_reduce({op}, {t.dtype})").all_reduce_here(t, op)
        self.wait()  # every earlier collective (same rank order of launches) first
        self.all_reduce(t, op)

    def broadcast(self, t: torch.Tensor, root: int = 0):
        if not self._words_ok(t):
            return self._inner(f"broadcast({t.dtype})").broadcast(t, root)
        self._guard()
        rid, off = self._loc(t, "broadcast")
        self._c.broadcast(rid, off, t, int(root), self.blocks, self._tmo_us)
        self.ops["broadcast"] += 1

    def gather(self, send: torch.Tensor, recv: Optional[torch.Tensor], root: int = 0):
        if not self._words_ok(send) or (recv is not None and not self._words_ok(recv)):
            return self._inner("gather").gather(send, recv, root)
        self._guard()
        rid, off = self._loc(send, "gather")
        self._c.gather(rid, off, send, recv if self.rank == root else None, int(root), self.blocks, self._tmo_us)
        self.ops["gather"] += 1

    def reduce_scatter(self, send: torch.Tensor, recv: torch.Tensor, op: str = "sum"):
        if not (self._words_ok(send) and self._words_ok(recv) and send.dtype == recv.dtype == torch.float32
                and op in _RED):
            return self._inner("reduce_scatter").reduce_scatter(send, recv, op)
        self._guard()
        rid, off = self._loc(send, "reduce_scatter")
        self._c.reduce_scatter(rid, off, send, recv, _RED[op], self.blocks, self._tmo_us)
        self.ops["reduce_scatter"] += 1

    def all_gather(self, send: torch.Tensor, recv: torch.Tensor):
        if not (self._words_ok(send) and self._words_ok(recv)):
            return self._inner("all_gather").all_gather(send, recv)
        self._guard()
        rid, off = self._loc(send, "all_gather")
        n = send.numel() * send.element_size() // 4
        if rid >= 0 and send.data_ptr() != recv.data_ptr() + self.rank * n * 4:
            # registered but not in place: the peers' inputs need not sit at this rank's offset
            # (e.g. arena[rank * n:]), so the input goes through the inbox instead
            rid, off = -1, 0
            self.ops["all_gather_bounced"] += 1
        self._c.all_gather(rid, off, send, recv, self.blocks, self._tmo_us)
        self.ops["all_gather"] += 1

    def synchronize(self):
        if self.inner is not None:
            self.inner.synchronize()
        elif self.side is not None:
            self.side.synchronize()

    def barrier(self):
        """Device barrier over the ranks (one peer-kernel launch), then a host wait for it."""
        if self.inner is not None:
            self.inner.barrier()
            return
        self._guard()
        with self.region():
            self._c.barrier(self.blocks, self._tmo_us)
        self.ops["barrier"] += 1
        self.wait()
        torch.cuda.current_stream(self.device).synchronize()

    @property
    def ipc_ops(self) -> int:
        return int(sum(self.ops.values()))

    def timed_out(self) -> bool:
        """A bounded peer wait gave up since the last call (clears the flag)."""
        return bool(self._c.take_timeout())

    def health_words(self):
        """(name, device address) of this communicator's error words (engine per-step health)."""
        return [(f"peer-collective wait timeout (IPC, rank {self.rank})", int(self._c.tmo_ptr()))]

    def check(self):
        if self.timed_out():
            raise RuntimeError(f"IPC collective on rank {self.rank}: a peer wait timed out (results invalid)")
        if self.inner is not None:
            self.inner.check()

    def close(self):
        if self.inner is not None:
            self.inner.close()
        else:
            self.synchronize()

    # ---- live agreement check ----
    def verify_all_reduce(self, t: torch.Tensor, rtol: float = 1e-6) -> dict:
        """Collective: all-reduce ``t`` (sum) through the peer kernel and check the result by a path
        that shares nothing with the device collectives -- three float64 checksums per rank (sum,
        a position-weighted sum, sum of magnitudes) through the store.  ``ok`` when every rank holds
        the same result, its checksums equal the sums of the inputs' to rounding (``rtol`` of the
        magnitude sum; an fp32 sum of W values is off by at most ~W 2^-24 of it), and no peer wait
        timed out.  A stale or torn read of a peer's memory (a cross-GPU visibility failure)
        changes the checksums by far more.  Every rank returns the same verdict.
        DPA_IPC_TEST_DISAGREE=1 (tests only) corrupts the last rank's result first."""
        n = t.numel()
        w = getattr(self, "_vw", None)
        if w is None or w.numel() < n:
            # weights 1 .. 1.875 by a multiplicative hash of the index: a permutation of elements
            # (a slice landing at the wrong offset) changes the weighted sum
            idx = torch.arange(n, device=self.device, dtype=torch.int64)
            w = self._vw = 1.0 + ((idx * 2654435761) % 8).double() / 8.0
        wt = w[:n]

        def sums(x):
            xd = x.double()
            return [float(xd.sum()), float((xd * wt).sum()), float(xd.abs().sum())]

        cin = sums(t)
        with self.region():
            self.all_reduce(t)
        self.wait()
        torch.cuda.synchronize(self.device)
        tmo = self.timed_out()
        if os.environ.get("DPA_IPC_TEST_DISAGREE") == "1" and self.rank == self.world - 1:
            t.view(-1)[0] += 1.0
        cout = sums(t)
        self._nreg += 1
        rows = [json.loads(v) for v in self._exchange(f"verify{self._nreg}", json.dumps([cin, cout, tmo]).encode())]
        same = all(r[1] == rows[0][1] for r in rows)
        scale = max(sum(r[0][2] for r in rows), 1e-30)
        err = max(abs(rows[0][1][k] - sum(r[0][k] for r in rows)) for k in range(2)) / scale
        ok = same and not any(r[2] for r in rows) and err <= rtol
        return {"ok": bool(ok), "ranks_identical": bool(same), "rel_err": err, "timed_out": any(r[2] for r in rows)}

    # ---- bootstrap check ----
    def _self_check(self) -> bool:
        """Exact-integer collectives through both input paths: a registered all-reduce (sum of
        rank + 1 and of a ramp, odd length: slice tails) and a bounced broadcast of rank 0's ramp.
        True when every element is exact and no wait timed out."""
        n = 4099
        t = torch.arange(n + 1, dtype=torch.float32, device=self.device)[:n] + float(self.rank + 1)
        self.register(t)
        b = torch.arange(1001, dtype=torch.float32, device=self.device) * (1.0 if self.rank == 0 else -1.0)
        with self.region():
            self.all_reduce(t)
            self.broadcast(b, 0)
        self.wait()
        torch.cuda.synchronize(self.device)
        if self.timed_out():
            return False
        W = self.world
        exp = torch.arange(n, dtype=torch.float32) * W + W * (W + 1) / 2
        return torch.equal(t.cpu(), exp) and torch.equal(b.cpu(), torch.arange(1001, dtype=torch.float32))
