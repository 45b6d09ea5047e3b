"""Gradient-synchronisation strategies — the reference's three DP modes, MI355X-first.

  mode "gather"    (main_gather.py:42-59)     grads → rank 0 (grouped send/recv into a W×n
                   buffer), mean-of-W kernel on rank 0, broadcast back (== scattering W copies).
  mode "allreduce" (main_all_reduce.py:45-48) all_reduce(SUM) per tensor, /W fused into SGD.
  mode "ddp"       (main_ddp.py:137)          DDP semantics: initial broadcast of params+buffers
                   from rank 0, BN buffers broadcast before every training forward, bucketed
                   all_reduce(SUM) overlapped with backward, /W fused into SGD.
  mode "zero1"     (new scope)                DDP semantics with a sharded optimizer step (ZeRO
                   stage 1): each bucket is reduce-scattered during backward, every rank updates
                   only its 1/W of the parameters (fused SGD on its slices), then the buckets are
                   all-gathered.  Same numerics as "ddp"; the optimizer's memory traffic is 1/W.

Differences from the reference, all by design:
* every mode works on contiguous slices of the flat grad arena (no per-step allocation, no
  stack/copy), and by default issues each bucket's collective on the comm stream as soon as the
  static backward schedule reports its layer done (``overlap=True``); ``overlap=False`` defers
  all collectives to after backward (the reference's blocking placement, for A/B comparison);
* buckets are cut at layer boundaries with an xGMI-sized cap (``bucket_mb``, default 10 MiB: the
  three 9 MiB [512,512,3,3] weights each get a bucket; the last-ready bucket is kept small so the
  exposed tail after backward is short) instead of DDP's 25 MiB/1 MiB;
* all modes broadcast rank 0's parameters (and momenta, when resuming) once at start (SURVEY
  §5.4), so replicas cannot silently fork; BN buffers only in the modes that share them (ddp/zero1);
* optionally (``DPA_FUSED_STEP=1``) the optimizer step is fused per bucket into backward: once a
  bucket's collective is issued AND the engine reports its parameters no longer read this step
  (``params_free``: dgrad of that layer enqueued), the fused SGD of that slice is queued behind the
  collective on the comm stream, so only the small tail bucket's collective and update follow
  backward.  Per-element SGD math is unchanged, so results are bitwise identical to the default
  single SGD launch after ``finish()`` — which measures faster on MI355X (see GradSync).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch

from ..utils.streams import DevEvent, StreamJoin
from .comm import Comm




class Bucket:
    __slots__ = ("names", "lo", "hi", "pending", "issued", "busy", "stepped", "free_ev", "free_sig")

    def __init__(self, names: List[str], lo: int, hi: int):
        self.names = list(names)
        self.lo, self.hi = lo, hi
        self.pending = set(names)   # gradients not yet produced this step
        self.busy = set(names)      # parameters still read by kernels not yet enqueued this step
        self.issued = False         # collective enqueued
        self.stepped = False        # optimizer step of this slice enqueued
        self.free_ev = None         # main-stream event after the last reader of the parameters
        self.free_sig = None        # ... or a later main-stream kernel's start signal (flag, value)

    @property
    def numel(self):
        return self.hi - self.lo


def plan_buckets(arena, ready_order: List[List[str]], bucket_mb: float, tail_mb: float = 2.0) -> List[Bucket]:
    """Greedy layer-aligned buckets in gradient-ready order.  ``bucket_mb <= 0`` → one bucket
    per tensor (the reference's per-parameter granularity)."""
    if bucket_mb <= 0:
        out = []
        for group in ready_order:
            for n in group:
                lo, hi = arena.span([n])
                out.append(Bucket([n], lo, hi))
        return out
    cap = bucket_mb * (1 << 20) / 4
    tail = tail_mb * (1 << 20) / 4
    groups = [(g, arena.span(g)) for g in ready_order]
    # the trailing (last-ready) groups form a small tail bucket
    tail_groups = []
    acc = 0
    while groups and acc + (groups[-1][1][1] - groups[-1][1][0]) <= tail and len(groups) > 1:
        g = groups.pop()
        acc += g[1][1] - g[1][0]
        tail_groups.insert(0, g)
    buckets, cur, cur_n = [], [], 0
    for g, (lo, hi) in groups:
        n = hi - lo
        if cur and cur_n + n > cap:
            buckets.append(cur)
            cur, cur_n = [], 0
        cur.append((g, (lo, hi)))
        cur_n += n
    if cur:
        buckets.append(cur)
    if tail_groups:
        buckets.append(tail_groups)
    out = []
    for b in buckets:
        names = [n for g, _ in b for n in g]
        lo, hi = arena.span(names)
        out.append(Bucket(names, lo, hi))
    # sanity: buckets must tile contiguous, non-overlapping ranges
    rng = sorted((b.lo, b.hi) for b in out)
    for (a0, a1), (b0, b1) in zip(rng, rng[1:]):
        assert a1 <= b0, "bucket ranges overlap"
    return out


class GradSync:
    mode = "none"

    # whether this mode's optimizer step can run per bucket inside backward (see module doc)
    fusable_step = True
    # whether BN buffers are kept equal across ranks (DDP broadcast_buffers).  Modes A/B keep per-rank
    # statistics: the start-up broadcast then sends only parameters/momenta, so a resumed run keeps
    # each rank's own running stats (identical at a fresh start anyway: same seed, same init).
    shared_buffers = False

    def __init__(self, engine, comm: Comm, bucket_mb: float = 0.0, overlap: bool = True, broadcast_init: bool = True,
                 tail_mb: float = 2.0):
        self.engine = engine
        self.comm = comm
        self.world = comm.world
        self.active = comm.name != "null"  # a real communicator (also a forced 1-rank one)
        self.overlap = overlap
        # DPA_FUSED_STEP: 0 (default: one SGD over the arena after backward) | 1 (per-bucket SGD
        # inside backward) | auto (per bucket with a real communicator).  Re-measured on MI355X after
        # the kernel-start-signal changes (1-rank RCCL, interleaved pairs): the per-bucket updates on
        # the comm stream delay the critical-path kernels by more than the ~32 us of update they
        # take off the tail: DDP 166.5k vs 168.0k img/s, per-tensor all-reduce mode (34 buckets)
        # 114-125k vs 154k (docs/PERF_NOTES.md).
        fused = os.environ.get("DPA_FUSED_STEP", "0")
        self.fuse_step = overlap and self.fusable_step and (fused == "1" or (fused == "auto" and self.active))
        self._cuda = engine.device.type == "cuda"
        order = [["fc1.weight", "fc1.bias"]] + [
            [f"{l.conv_key}.weight", f"{l.conv_key}.bias", f"{l.bn_key}.weight", f"{l.bn_key}.bias"]
            for l in reversed(engine.spec.convs)]
        self.bucket_mb, self.tail_mb = bucket_mb, tail_mb
        self.buckets = plan_buckets(engine.grads, order, bucket_mb, tail_mb)
        self._by_name: Dict[str, Bucket] = {n: b for b in self.buckets for n in b.names}
        self._join = StreamJoin() if self._cuda else None
        if self._cuda:
            for b in self.buckets:
                b.free_ev = DevEvent()
        self.issued_bytes = 0
        # The last bucket's collective goes on the stream that reports it (the main stream, right
        # after backward) once that stream has waited for the comm stream: the all-reduce then needs
        # no hop there and no hop back before the update (1-rank RCCL trace: ~34 us of step tail in
        # two cross-stream hops).
        self.tail_here = (self._cuda
                          and type(self).reduce_bucket_here is not GradSync.reduce_bucket_here)
        self._joined = False
        self._main = None
        # optional utils.profiling.EventProbe: marks b{i}_start / b{i}_end around each bucket's
        # collective on the comm stream (bench diagnostic phase only)
        self.probe = None
        self._index = {id(b): i for i, b in enumerate(self.buckets)}
        if self.active and self._cuda:  # the arenas every collective of this strategy moves
            e = engine
            comm.prepare([e.grads.flat, e.params.flat, e.mom.flat, e.buffers.flat, e.nbt])
            # device error words of the communicator (peer-collective timeouts) join the engine's
            # per-step health snapshot
            if hasattr(engine, "add_health_word"):
                for nm, addr in getattr(comm, "health_words", lambda: [])():
                    engine.add_health_word(nm, addr)
        if broadcast_init and self.active:
            self.broadcast_state()

    # -- state broadcast (DDP ctor semantics; torch distributed.py:862-871) --
    def broadcast_state(self):
        e = self.engine
        with self.comm.region():
            self.comm.broadcast(e.params.flat, 0)
            if self.shared_buffers:
                self.comm.broadcast(e.buffers.flat, 0)
                self.comm.broadcast(e.nbt, 0)
            if e.steps_taken > 0:
                self.comm.broadcast(e.mom.flat, 0)
        self.comm.wait()
        e.refresh_weight_planes()

    def prepare_checkpoint(self):
        """Collective hook before every rank writes its checkpoint: make the local optimizer state
        complete (a no-op except for sharded optimizer state)."""

    def pre_forward(self):
        """Called before the training forward.  May return a callable that the engine invokes
        right before the first read of the BN buffers (so a buffer broadcast overlaps the first
        conv instead of stalling the step)."""
        return None

    def begin_step(self):
        for b in self.buckets:
            b.pending = set(b.names)
            b.busy = set(b.names)
            b.issued = False
            b.stepped = False
            b.free_sig = None
        self._joined = False
        self._main = torch.cuda.current_stream(self.engine.device) if self._cuda else None

    def grad_ready(self, names: List[str]):
        for n in names:
            b = self._by_name.get(n)
            if b is None:
                continue
            b.pending.discard(n)
            if b.pending:
                continue
            if self.active and self.overlap and not b.issued:
                self._issue(b)
            self._maybe_step(b)

    def params_free(self, names: List[str], signal=None):
        """Engine hook (main stream current): no kernel of this step still to be enqueued reads
        these parameters.  ``signal``: a kernel-start signal of a later main-stream kernel (engine
        forward_backward); the update waits on it instead of an event recorded here."""
        if not self.fuse_step:
            return
        for n in names:
            b = self._by_name.get(n)
            if b is None or n not in b.busy:
                continue
            b.busy.discard(n)
            if b.busy:
                continue
            b.free_sig = signal
            if b.free_ev is not None and signal is None:
                b.free_ev.record(torch.cuda.current_stream(self.engine.device))
            self._maybe_step(b)

    def _maybe_step(self, b: Bucket):
        """Enqueue the fused SGD of bucket b once its gradients are final (collective issued) and
        its parameters are free.  Runs on the comm stream behind the collective; for a single rank
        on the engine's wgrad stream (else inline on the current stream)."""
        if not self._step_ready(b) or (self.active and not b.issued):
            return
        if self.active:
            with self.comm.region():  # comm stream: behind the collective, after the triggering stream
                self._step_here(b)
            return
        b.stepped = True
        scale = self.grad_scale()
        s = self.engine.wstream if self._cuda else None
        if s is None:
            self.engine.sgd_step(scale, b.lo, b.numel)
            return
        self._join(s, torch.cuda.current_stream(self.engine.device))
        with torch.cuda.stream(s):
            self._wait_free(b)
            self.engine.sgd_step(scale, b.lo, b.numel)

    def _step_ready(self, b: Bucket) -> bool:
        return self.fuse_step and not b.stepped and not b.pending and not b.busy

    def _step_here(self, b: Bucket):
        """The bucket's SGD on the current stream (the comm stream, inside a region), after the
        main-stream event that follows the last reader of its parameters."""
        b.stepped = True
        self._wait_free(b)
        self.engine.sgd_step(self.grad_scale(), b.lo, b.numel)

    def _wait_free(self, b: Bucket):
        """Order the current stream after the last reader of b's parameters."""
        if b.free_sig is not None:
            self.engine.wait_signal(b.free_sig)
        elif b.free_ev is not None:
            b.free_ev.wait(torch.cuda.current_stream(self.engine.device))

    def _issue(self, b: Bucket):
        b.issued = True
        self.issued_bytes += 4 * b.numel
        if (self.tail_here and not self.fuse_step and self.probe is None and self._main is not None
                and all(o.issued for o in self.buckets)
                and torch.cuda.current_stream(self.engine.device) == self._main):
            self.reduce_bucket_here(b)  # the last bucket: on the main stream (see __init__)
            self._joined = True
            return
        with self.comm.region():
            if self.probe is not None:
                self.probe.mark(f"b{self._index[id(b)]}_start")
            self.reduce_bucket(b)
            if self.probe is not None:
                self.probe.mark(f"b{self._index[id(b)]}_end")
            if self._step_ready(b):  # parameters already free: update in the same region (one join)
                self._step_here(b)

    def reduce_bucket(self, b: Bucket):
        raise NotImplementedError

    def reduce_bucket_here(self, b: Bucket):
        """reduce_bucket ordered on the current stream (modes whose collective is one all-reduce)."""
        raise NotImplementedError

    def finish(self) -> float:
        """Issue whatever is left, make the compute stream wait for the comm stream, and return
        the scale the optimizer must apply to the synced grads."""
        if not self.active:
            if self.fuse_step and self._cuda and self.engine.wstream is not None:
                self._join(torch.cuda.current_stream(self.engine.device), self.engine.wstream)
            return 1.0
        for b in self.buckets:
            if not b.issued:
                self._issue(b)
            self._maybe_step(b)
        if not self._joined:  # (the tail collective on the main stream already joined the comm stream)
            self.comm.wait()
        return self.grad_scale()

    def grad_scale(self) -> float:
        return 1.0

    def update(self, grad_scale: float):
        """Apply the optimizer step to the synchronised gradients (the whole arena by default;
        with the fused step only slices whose update was not already queued during backward)."""
        if not self.fuse_step:
            self.engine.sgd_step(grad_scale)
            return
        for b in self.buckets:
            if not b.stepped:
                b.stepped = True
                self.engine.sgd_step(grad_scale, b.lo, b.numel)


class GatherScatterSync(GradSync):
    """Mode A: gather → mean on rank 0 → broadcast (main_gather.py:42-59)."""

    mode = "gather"

    def __init__(self, engine, comm, bucket_mb: float = 0.0, overlap: bool = True, broadcast_init: bool = True,
                 tail_mb: float = 2.0):
        super().__init__(engine, comm, bucket_mb, overlap, broadcast_init, tail_mb)
        self._recv = None
        if comm.rank == 0 and self.active:
            mx = max(b.numel for b in self.buckets)
            self._recv = torch.empty(comm.world * mx, device=engine.device, dtype=torch.float32)

    def reduce_bucket(self, b: Bucket):
        g = self.engine.grads.flat[b.lo:b.hi]
        recv = self._recv[: self.world * b.numel] if self._recv is not None else None
        self.comm.gather(g, recv, 0)
        if self.comm.rank == 0:
            self.engine.K.mean_of_w(recv, g, self.world)
        self.comm.broadcast(g, 0)


class AllReduceSync(GradSync):
    """Mode B: per-tensor all_reduce(SUM), then grad /= W (fused into SGD)."""

    mode = "allreduce"

    def reduce_bucket(self, b: Bucket):
        self.comm.all_reduce(self.engine.grads.flat[b.lo:b.hi], "sum")

    def reduce_bucket_here(self, b: Bucket):
        self.comm.all_reduce_here(self.engine.grads.flat[b.lo:b.hi], "sum")

    def grad_scale(self) -> float:
        return 1.0 / self.world


class DDPSync(GradSync):
    """Mode C: DistributedDataParallel semantics on RCCL.

    One intentional difference from torch DDP: rank 0's BN running statistics are broadcast right
    after each training forward (under the backward) instead of before the next forward, so after
    the last training step every replica already holds rank 0's statistics — which torch DDP only
    establishes at the first eval forward.  Eval results are identical; a per-rank checkpoint taken
    at that point holds rank 0's statistics on every rank."""

    mode = "ddp"

    def __init__(self, engine, comm, bucket_mb: float = 10.0, overlap: bool = True, broadcast_init: bool = True,
                 broadcast_buffers: bool = True, tail_mb: float = 2.0):
        self.shared_buffers = broadcast_buffers
        super().__init__(engine, comm, bucket_mb, overlap, broadcast_init, tail_mb)
        self.broadcast_buffers = broadcast_buffers
        self._bufs_fresh = False  # replicas hold rank 0's running stats (sent after the last forward)
        self._bufs_sent = False   # ... sent during the current step
        self._sig_bufs = False    # this step's broadcast waits on a kernel-start signal

    # DDP._sync_buffers (torch nn/parallel/distributed.py:2178): rank 0's BN running stats
    # overwrite every replica's before each training forward.  Nothing touches the running stats
    # between the end of one training forward and the start of the next, so the broadcast is
    # issued as soon as this step's forward is done (first grad_ready), where it runs on the comm
    # stream under the backward; the next forward then finds the replicas already in sync and
    # needs no stream hop.  The num_batches_tracked counters advance identically on every replica
    # after the start-up broadcast, so they are not re-sent.
    #
    # With the engine's kernel-start signals the broadcast waits on the signal that the first BN
    # backward raises (forward and head complete) instead of an event recorded on the compute
    # stream: it is issued from the first params_free that carries a signal (fc1 for VGG).
    def _send_buffers(self, signal=None):
        with self.comm.region(join=signal is None):
            if signal is not None:
                self.engine.wait_signal(signal)
            self.comm.broadcast(self.engine.buffers.flat, 0)
        self._bufs_sent = self._bufs_fresh = True

    def _post_forward_send(self) -> bool:
        return self.active and self.broadcast_buffers and not self._bufs_sent

    def begin_step(self):
        super().begin_step()
        self._bufs_sent = False
        # a signal will come with the head's params_free (engine forward_backward, eager steps)
        e = self.engine
        self._sig_bufs = (getattr(e, "ksignal", False) and getattr(e, "free_signal", False)
                          and not torch.cuda.is_current_stream_capturing())

    def grad_ready(self, names: List[str]):
        if self._post_forward_send() and not self._sig_bufs:
            self._send_buffers()  # the engine reports gradients only once the forward is done
        super().grad_ready(names)

    def params_free(self, names: List[str], signal=None):
        if self._post_forward_send() and (signal is not None or not self._sig_bufs):
            self._send_buffers(signal)
        super().params_free(names, signal)

    def finish(self) -> float:
        if self._post_forward_send():  # no signal arrived (e.g. a caller without params_free)
            self._send_buffers()
        return super().finish()

    def pre_forward(self):
        if not self.active or not self.broadcast_buffers:
            return None
        if self._bufs_fresh:  # already broadcast after the previous training forward
            self._bufs_fresh = False
            return None
        self._send_buffers()  # first forward, or a caller that bypasses grad_ready
        return self.comm.wait

    def reduce_bucket(self, b: Bucket):
        self.comm.all_reduce(self.engine.grads.flat[b.lo:b.hi], "sum")

    def reduce_bucket_here(self, b: Bucket):
        self.comm.all_reduce_here(self.engine.grads.flat[b.lo:b.hi], "sum")

    def grad_scale(self) -> float:
        return 1.0 / self.world


class ZeroSync(DDPSync):
    """ZeRO-1 on the flat arenas: reduce_scatter(SUM) per bucket during backward (in place: the
    rank's shard of the bucket receives the sum), SGD on the owned shards only, all_gather of
    every bucket's parameters, then one split kernel refreshes the bf16 weight planes.  Bucket
    spans are multiples of 64 elements, so W | 16 keeps every shard float4-aligned."""

    mode = "zero1"
    fusable_step = False  # the update is sharded (owned slices after reduce-scatter, then all-gather)
    reduce_bucket_here = GradSync.reduce_bucket_here  # (a reduce-scatter: every bucket on the comm stream)

    def __init__(self, engine, comm, bucket_mb: float = 10.0, overlap: bool = True, broadcast_init: bool = True,
                 broadcast_buffers: bool = True, tail_mb: float = 2.0):
        super().__init__(engine, comm, bucket_mb, overlap, broadcast_init, broadcast_buffers, tail_mb)
        if self.active:
            for b in self.buckets:
                if b.numel % (4 * self.world):
                    raise ValueError(f"zero1: bucket of {b.numel} elements does not split into 4-aligned shards "
                                     f"over {self.world} ranks")

    def broadcast_state(self):
        """Parameters (and BN buffers) from rank 0, but NOT momenta: under ZeRO-1 every rank updates
        only its own shards' momentum, so rank 0's copy of the other shards is stale.  A resumed
        rank holds the complete momentum arena already (``prepare_checkpoint`` all-gathers the
        shards before each save)."""
        e = self.engine
        with self.comm.region():
            self.comm.broadcast(e.params.flat, 0)
            if self.shared_buffers:
                self.comm.broadcast(e.buffers.flat, 0)
                self.comm.broadcast(e.nbt, 0)
        self.comm.wait()
        e.refresh_weight_planes()

    def prepare_checkpoint(self):
        """All-gather every bucket's owned momentum shards so each rank's arena (and checkpoint)
        holds the full, current SGD state."""
        if not self.active:
            return
        e = self.engine
        with self.comm.region():
            for b in self.buckets:
                lo, sb = self._shard(b)
                self.comm.all_gather(e.mom.flat[lo:lo + sb], e.mom.flat[b.lo:b.hi])
        self.comm.wait()

    def _shard(self, b: Bucket):
        sb = b.numel // self.world
        lo = b.lo + self.comm.rank * sb
        return lo, sb

    def reduce_bucket(self, b: Bucket):
        g = self.engine.grads.flat
        lo, sb = self._shard(b)
        self.comm.reduce_scatter(g[b.lo:b.hi], g[lo:lo + sb], "sum")

    def update(self, grad_scale: float):
        e = self.engine
        if not self.active:
            e.sgd_step(grad_scale)
            return
        for b in self.buckets:  # the owned shards (compute stream, after finish()'s wait)
            lo, sb = self._shard(b)
            e.sgd_step(grad_scale, lo, sb)
        with self.comm.region():
            for b in self.buckets:
                lo, sb = self._shard(b)
                self.comm.all_gather(e.params.flat[lo:lo + sb], e.params.flat[b.lo:b.hi])
        self.comm.wait()
        e.refresh_weight_planes()


MODES = {"gather": GatherScatterSync, "allreduce": AllReduceSync, "ddp": DDPSync, "zero1": ZeroSync}
DEFAULT_BUCKET_MB = {"gather": 0.0, "allreduce": 0.0, "ddp": 10.0, "zero1": 10.0}


def make_sync(mode: str, engine, comm: Comm, bucket_mb: Optional[float] = None, overlap: bool = True,
              broadcast_init: bool = True, tail_mb: float = 2.0) -> GradSync:
    cls = MODES[mode]
    bmb = DEFAULT_BUCKET_MB[mode] if bucket_mb is None else bucket_mb
    return cls(engine, comm, bmb, overlap, broadcast_init, tail_mb=tail_mb)
