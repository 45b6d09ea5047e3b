"""Headline benchmark: VGG-11 / CIFAR-10-shaped training throughput (images/sec, whole job).

BASELINE.json metric: "images/sec whole-node VGG-11 CIFAR-10 at 1/2/4/8 MI355X; scaling efficiency".
Config is the reference's: VGG-11 (BN), batch 256 per rank (weak scaling), SGD(0.1, 0.9, wd 1e-4),
fp32-grade compute (the reference trains in fp32), synthetic CIFAR-shaped data on device, random
init (seed 1).  Every timed step is a full training step: on-device augmentation of the batch,
forward, loss, backward, gradient synchronisation (DDP mode by default: bucketed RCCL all-reduce
overlapped with backward + BN-buffer broadcast), fused SGD update.

    python bench.py [--gpus N] [--steps 50] [--warmup 10] [--mode ddp|allreduce|gather|zero1]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W
    python bench.py --profile            # the same run under rocprofv3 --kernel-trace --stats

``--gpus N`` without torchrun starts N local ranks itself (parallel/spawn.py: fresh child
processes, the parent never touches the GPU).  For N > 1, rank 0 first times the same step alone
(``--solo-steps``, no communicator; the other ranks wait) so the JSON line carries a same-run
scaling efficiency; after the timed steps a short diagnostic phase records the communication left
exposed after backward and each bucket's collective time with timing events (kept out of the
timed region), and the parameter arenas are compared across ranks.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_pytorch_amd.data import DeviceLoader, ShardSampler, synthetic_cifar  # noqa: E402
from distributed_pytorch_amd.engine import VGGEngine  # noqa: E402
from distributed_pytorch_amd.graph_step import GraphedStep  # noqa: E402
from distributed_pytorch_amd.parallel import NullComm, init_env, make_sync  # noqa: E402
from distributed_pytorch_amd.parallel.ipc import IpcComm  # noqa: E402
from distributed_pytorch_amd.parallel.spawn import is_spawned_child  # noqa: E402
from distributed_pytorch_amd.utils import benchlib  # noqa: E402
from distributed_pytorch_amd.utils.profiling import EventProbe, step_comm_report  # noqa: E402

BASELINE_METRIC = "images/sec whole-node VGG-11 CIFAR-10 at 1/2/4/8 MI355X; scaling efficiency"  # BASELINE.json
# BASELINE.md (reference harness measured on CPU — the only numbers the reference has)
BASELINE_IMG_S = {1: 397.8, 2: 601.8}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch (reference: 256 per node)")
    ap.add_argument("--mode", default="ddp", choices=["ddp", "allreduce", "gather", "zero1"])
    ap.add_argument("--model", default="VGG11")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "ipc", "torch", "gloo"],
                    help="ipc: every collective on the peer-memory kernels (one node; ranks may share a GPU)")
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--graph", default="off", choices=["auto", "off", "on"],
                    help="single GPU: replay the captured step as a HIP graph (graph_step.py; auto = on with an "
                         "eager fallback).  Off by default: same throughput on MI355X (host enqueue 0.67 -> 0.27 "
                         "ms hides behind 1.7 ms of GPU work) and the graph executor reorders the two-stream "
                         "backward")
    ap.add_argument("--impl", default="h2", choices=["fp32", "x3", "h2", "bf16"],
                    help="conv kernels: h2 = fp32-grade results from fp16 matrix cores (fp16 pairs of scaled "
                         "operands, 3 products; default) | x3 = fp32-grade from bf16 matrix cores (3 planes, "
                         "6 products) | fp32 = fp32 MFMA | bf16 = mixed precision.  h2 and x3 are pinned "
                         "against fp64 at this exact config by tests/test_parity256_gpu.py")
    ap.add_argument("--solo-steps", type=int, default=None,
                    help="N>1: steps rank 0 times alone first (same-run 1-GPU figure; 0 = skip; default "
                         "min(steps, 30))")
    ap.add_argument("--diag-steps", type=int, default=5,
                    help="diagnostic steps after the timed region (exposed comm / per-bucket times; 0 = off)")
    ap.add_argument("--comm-tune", default="auto", choices=["auto", "off"],
                    help="N>1, ddp/allreduce modes: in the warmup, time a few gradient-sync plans (bucket size, "
                         "tail bucket, per-bucket update inside backward) on the real fabric and keep the fastest "
                         "(max over ranks, so every rank picks the same plan); off = --bucket-mb / defaults")
    ap.add_argument("--comm-tune-steps", type=int, default=8, help="timed steps per plan and repetition")
    ap.add_argument("--comm-tune-budget", type=float, default=60.0,
                    help="wall-clock seconds the comm tuner may take in all (agreed over ranks; plans not reached "
                         "are skipped, the default plan stays the fallback)")
    ap.add_argument("--ipc", default="off", choices=["auto", "on", "off"],
                    help="N>1 on one node: collectives on the peer-memory kernels (parallel/ipc.py). auto = "
                         "extra comm-tuner plans; on = always (any --comm; several ranks may share a GPU); off "
                         "(default): ranks sharing one GPU through them are not run-to-run reproducible "
                         "(docs/PERF_NOTES.md round 5), so the default path is RCCL")
    ap.add_argument("--ipc-blocks", default="32,16,64",
                    help="workgroups per rank of the peer-memory collectives the comm tuner tries (comma list; the "
                         "first is the --ipc on / --comm ipc default unless DPA_IPC_BLOCKS is set)")
    ap.add_argument("--rccl-channels", default="16,8",
                    help="N>1 with the native RCCL communicator: channel (workgroup) budgets the comm tuner also "
                         "tries, each on its own communicator (comma list; 'off' = RCCL's default only)")
    ap.add_argument("--profile", action="store_true",
                    help="re-run this command under rocprofv3 --kernel-trace --stats (prints the command)")
    ap.add_argument("--profile-dir", default="gpurun_out/prof")
    ap.add_argument("--launch-timeout", type=float, default=1800.0, help="wall-clock limit of a self-launched job")
    ap.add_argument("--torch-baseline", type=int, default=0, metavar="STEPS",
                    help="1 GPU: first time STEPS steps of stock PyTorch-ROCm eager fp32 training of the same model "
                         "and batch (tools/torch_baseline.py, in a child process on this GPU) and report "
                         "vs_torch_eager_fp32 from this same run (0 = off)")
    return ap.parse_args(argv)


def build(a, dev, rank, world, comm):
    engine, sync, batches = build_parts(a, dev, rank, world, comm)
    return engine, sync, batches()


def build_parts(a, dev, rank, world, comm):
    """(engine, sync, batches): ``batches()`` starts a fresh endless iterator over the sharded
    synthetic set (the warmup tuner draws its own, so the timed run sees the same data)."""
    train = synthetic_cifar(50000, 0)
    sampler = ShardSampler(len(train), world, rank, shuffle=True, seed=0)
    loader = DeviceLoader(train, a.batch, dev, sampler=sampler, train=True, seed=7919 + rank, drop_last=True)
    engine = VGGEngine(a.model, dev, max_batch=a.batch, impl=a.impl)
    engine.init_parameters(seed=1)
    sync = make_sync(a.mode, engine, comm, bucket_mb=a.bucket_mb, overlap=not a.no_overlap,
                     tail_mb=float(os.environ.get("DPA_TAIL_MB", "2.0")))  # (env: A/B of the tail bucket)

    def batches():
        ep = 0
        while True:
            loader.set_epoch(ep)
            yield from loader  # drop_last: every step has the full per-GPU batch
            ep += 1

    return engine, sync, batches


def make_step(engine, sync, it, graphed=None, probe=None):
    def step():
        x, t = next(it)
        if graphed is not None:
            graphed.run(x, t)
            return
        sync.begin_step()
        engine.forward_backward(x, t, grad_ready=sync.grad_ready, pre_forward=sync.pre_forward,
                                params_free=sync.params_free)
        if probe is not None:
            probe.mark("bwd_end")
        sync.update(sync.finish())
        if probe is not None:
            probe.mark("step_end")
        engine.finish_step()

    if probe is None:
        return step

    orig_finish = sync.finish

    def finish():  # mark when the compute stream has caught up with the comm stream
        s = orig_finish()
        probe.mark("synced")
        return s

    sync.finish = finish
    return step


def comm_plans(a, rccl: bool = False, ipc: bool = False):
    """Candidate gradient-sync plans (bucket_mb, tail_mb, per-bucket update, rccl_channels,
    ipc_blocks) for the warmup tuner.  Per-tensor modes keep their granularity (the reference's semantics)
    and only try the update placement; an explicit --bucket-mb pins the bucket size.  With a native
    RCCL communicator (``rccl``) the default plan is also tried on communicators limited to
    ``--rccl-channels`` workgroups: fewer RCCL workgroups leave more CUs to the backward the
    collectives overlap (channels 0 = the communicator RCCL sized itself).  ``ipc``: the default
    plan is also tried with every collective on the peer-memory kernels (parallel/ipc.py), at each of
    the ``--ipc-blocks`` workgroup budgets."""
    fixed = a.bucket_mb
    if a.mode == "ddp":
        sizes = [fixed] if fixed is not None else [10.0, 25.0, 5.0]
        plans = [(b, 2.0, False, 0, False) for b in sizes] + [(sizes[0], 2.0, True, 0, False),
                                                               (sizes[0], 0.4, False, 0, False)]
    elif a.mode == "allreduce":
        plans = [(fixed, 2.0, False, 0, False), (fixed, 2.0, True, 0, False)]
    else:
        plans = []
    if plans and rccl:
        plans += [plans[0][:3] + (c, False) for c in channel_budgets(a)]
    if plans and ipc:  # p[4]: the peer kernels' workgroups per rank (0: no peer kernels)
        plans += [plans[0][:3] + (0, b) for b in ipc_block_budgets(a)]
    seen, out = set(), []
    for p in plans:
        if p not in seen:
            seen.add(p)
            out.append(p)
    return out


def ipc_block_budgets(a):
    """Workgroups per rank the tuner tries for the peer-memory collectives (``--ipc-blocks``)."""
    return [int(b) for b in a.ipc_blocks.split(",") if int(b) > 0]


def channel_budgets(a):
    """RCCL channel budgets the tuner tries besides the default (``--rccl-channels``: a comma list,
    'off' = none; DPA_RCCL_CHANNELS pins the main communicator's budget instead)."""
    if a.rccl_channels == "off" or os.environ.get("DPA_RCCL_CHANNELS"):
        return []
    return [int(c) for c in a.rccl_channels.split(",") if int(c) > 0]


def comm_for_channels(ctx, dev, channels: int, cache: dict):
    """A communicator over the same ranks limited to ``channels`` RCCL workgroups (0: ctx.comm)."""
    if channels == 0:
        return ctx.comm
    if channels not in cache:
        from distributed_pytorch_amd.parallel.comm import RcclComm

        store = ctx.store if ctx.store is not None else torch.distributed.distributed_c10d._get_default_store()
        cache[channels] = RcclComm(ctx.rank, ctx.world, dev, store=store, tag=f"dpa_rccl_uid_ch{channels}",
                                   channels=channels)
    return cache[channels]


def ipc_possible(ctx, dev) -> bool:
    """Every rank on this node and on a GPU: the peer-memory all-reduce can map the peers."""
    return (dev.type == "cuda" and ctx.world > 1
            and int(os.environ.get("LOCAL_WORLD_SIZE", ctx.world)) == ctx.world and ctx.world <= 8)


def ipc_comm(ctx, dev, engine, cache: dict, blocks: int = 0):
    """The peer-memory communicator over ctx.comm with the engine's arenas registered (collective).
    Plans with different workgroup budgets share it (``blocks`` is a per-collective launch size)."""
    if "ipc" not in cache:
        store = ctx.store if ctx.store is not None else torch.distributed.distributed_c10d._get_default_store()
        c = IpcComm(ctx.comm, store, dev, timeout_s=20.0)
        c.prepare([engine.grads.flat, engine.params.flat, engine.mom.flat, engine.buffers.flat, engine.nbt])
        cache["ipc"] = c
    return cache["ipc"]


def ipc_live_checks(ipc, engine, checks: list):
    """After a diagnostic step: all-reduce the live gradient arena once more through the peer kernel
    and check it through the store (IpcComm.verify_all_reduce); the verdicts go into the JSON."""
    checks.append(ipc.verify_all_reduce(engine.grads.flat))


def _test_drop(rank: int, idx: int) -> bool:
    """Test hook: DPA_TEST_TUNE_DROP=rank:plan makes that rank fail to set up that plan."""
    spec = os.environ.get("DPA_TEST_TUNE_DROP")
    if not spec:
        return False
    r, i = (int(v) for v in spec.split(":"))
    return r == rank and i == idx


def tune_comm(a, engine, sync, ctx, dev, batches):
    """Warmup-phase choice among ``comm_plans``: each plan runs ``--comm-tune-steps`` steps per
    repetition (2 repetitions, interleaved); the score of a plan is its best repetition's time,
    each repetition's time being the max over ranks, so every rank picks the same plan.  Returns
    (sync, report).  Gradient-sync plans change only where and when collectives and the update
    run: the numerics of every plan are identical (bitwise, tests/test_multirank_gpu.py).  The
    tuning steps draw their own batches and the training state is restored afterwards, so the
    run that follows is the same as without tuning.

    First-contact safety on a real multi-GPU node: a plan's communicator is
    created only when that plan is first timed (its init time, max over ranks, is reported); the
    whole tuner runs under ``--comm-tune-budget`` seconds of wall clock, agreed over the ranks
    (``all_max``) before every plan, so every rank stops at the same plan -- plans not timed are
    not candidates and the default plan (always timed first) stays the fallback; a plan that
    fails to set up on ANY rank is dropped on every rank; the communicators of the plans not
    chosen are destroyed on every rank in the same order after a barrier."""
    from distributed_pytorch_amd.parallel.comm import RcclComm

    if isinstance(ctx.comm, IpcComm):  # --ipc on: the transport is fixed
        return sync, None
    plans = comm_plans(a, rccl=isinstance(ctx.comm, RcclComm) and ctx.world > 1,
                       ipc=a.ipc == "auto" and ipc_possible(ctx, dev))
    if ctx.world <= 1 or a.comm_tune == "off" or len(plans) < 2 or a.no_overlap:
        return sync, None
    t_tune = time.perf_counter()
    it = batches()
    snap = [t.clone() for t in (engine.params.flat, engine.mom.flat, engine.buffers.flat, engine.nbt,
                                engine.loss_accum)]
    steps_taken = engine.steps_taken
    syncs, comms, init_s = {}, {}, {}
    all_plans = list(plans)
    dropped = []

    def setup(p) -> bool:
        """Create plan p's communicator and sync (lazily); False (on every rank) if it failed anywhere."""
        if p in syncs:
            return True
        err, t0 = None, time.perf_counter()
        key = "ipc" if p[4] else p[3]
        try:
            if _test_drop(ctx.rank, all_plans.index(p)):
                raise RuntimeError("injected set-up failure (DPA_TEST_TUNE_DROP)")
            comm = ipc_comm(ctx, dev, engine, comms) if p[4] else comm_for_channels(ctx, dev, p[3], comms)
        except RuntimeError as e:
            err = e
        dt = ctx.all_max(time.perf_counter() - t0)
        name = "ipc" if p[4] else f"ch{p[3]}"
        if key != 0 and name not in init_s:
            init_s[name] = round(dt, 3)
        # a plan is dropped on EVERY rank if its communicator failed on ANY rank (a rank-local
        # failure must not leave the ranks with different plan lists: mismatched collectives hang)
        if ctx.all_max(1.0 if err is not None else 0.0) > 0:
            print(f"[rank {ctx.rank}] comm tuner: no communicator for plan {p} ({err or 'failed on a peer'})",
                  flush=True)
            dropped.append(p)
            if key != 0:
                comms.pop(key, None)
            return False
        s = make_sync(a.mode, engine, comm, bucket_mb=p[0], overlap=True, broadcast_init=False, tail_mb=p[1])
        s.fuse_step = p[2] and s.fusable_step
        syncs[p] = s
        return True

    n = max(1, a.comm_tune_steps)
    score = {}
    budget_hit = False
    for _rep in range(2):
        for p in list(plans):
            # the budget check is agreed (max over ranks): every rank stops before the same plan;
            # the default plan's first repetition always runs
            if score and ctx.all_max(time.perf_counter() - t_tune) > a.comm_tune_budget:
                budget_hit = True
                break
            if not setup(p):
                plans.remove(p)
                continue
            if p[4]:
                comms["ipc"].blocks = p[4]
            step = make_step(engine, syncs[p], it)
            for _ in range(2):
                step()
            benchlib.device_barrier(ctx, dev)
            t0 = time.perf_counter()
            for _ in range(n):
                step()
            benchlib.device_barrier(ctx, dev)
            el = ctx.all_max(time.perf_counter() - t0) / n * 1e3
            score[p] = min(score.get(p, el), el)
        if budget_hit:
            break
    plans = [p for p in plans if p in score]
    # a plan whose peer-memory waits timed out (any rank), or whose all-reduce of the real gradient
    # arena fails the store-side agreement check (IpcComm.verify_all_reduce: same verdict on every
    # rank), is disqualified
    ipc_check = None
    if "ipc" in comms:
        bad = ctx.all_max(1.0 if comms["ipc"].timed_out() else 0.0) > 0
        if not bad:
            ipc_check = comms["ipc"].verify_all_reduce(engine.grads.flat)
            bad = not ipc_check["ok"]
        if bad:
            print(f"[rank {ctx.rank}] comm tuner: IPC all-reduce timed out or disagreed ({ipc_check}); plan dropped",
                  flush=True)
            plans = [p for p in plans if not p[4]]
    # the first plan is the default: another one must beat it by 1 % (run-to-run noise of a few
    # steps), so the choice does not flap between equivalent plans
    best = min(plans, key=lambda p: score[p])
    if all_plans[0] in score and score[best] > 0.99 * score[all_plans[0]]:
        best = all_plans[0]
    benchlib.device_barrier(ctx, dev)
    for dst, src in zip((engine.params.flat, engine.mom.flat, engine.buffers.flat, engine.nbt, engine.loss_accum),
                        snap):
        dst.copy_(src)
    engine.steps_taken = steps_taken
    engine.refresh_weight_planes()
    engine._eval_dirty = True
    for sy in syncs.values():
        if hasattr(sy, "_bufs_fresh"):
            sy._bufs_fresh = False  # the next forward broadcasts rank 0's (restored) buffers again
    report = {"chosen": {"bucket_mb": best[0], "tail_mb": best[1], "per_bucket_update": best[2],
                         "rccl_channels": best[3] or None, "ipc_blocks": best[4] or None},
              "ipc_check": ipc_check,
              "budget_s": a.comm_tune_budget, "budget_hit": budget_hit,
              "untimed_plans": len(all_plans) - len(score) - len(dropped), "dropped_plans": len(dropped),
              # communicators the tuner created (max over ranks), the run's main one excluded
              "comm_init_s": init_s,
              "ms_per_step": {f"b{p[0]}_t{p[1]}_{'fused' if p[2] else 'after'}" + (f"_ch{p[3]}" if p[3] else "")
                              + (f"_ipc{p[4]}" if p[4] else ""): round(score[p], 4) for p in plans}}
    if best[4]:  # the peer-memory communicator carries the run from here on
        ctx.comm = comms.pop("ipc")
        ctx.comm.blocks = best[4]
    elif best[3]:  # the bounded communicator carries the run from here on (and the replica check)
        ctx.comm = comms.pop(best[3])
    chosen = syncs[best]
    # the unchosen communicators: drained, then destroyed on every rank in the same order
    for c in comms.values():
        c.synchronize()
    benchlib.device_barrier(ctx, dev)
    for k in sorted(comms, key=str):
        c = comms[k]
        if hasattr(c, "close"):
            c.close()
    syncs.clear()
    comms.clear()
    gc.collect()
    # the whole tuner (communicator creation, every plan, the agreement check), max over ranks
    report["tune_seconds"] = round(ctx.all_max(time.perf_counter() - t_tune), 3)
    if ctx.rank == 0:
        print(f"[bench] comm tuner: {report['tune_seconds']} s, chosen {report['chosen']}, "
              f"communicator init {init_s or '-'}, budget hit {budget_hit}", file=sys.stderr, flush=True)
    return chosen, report


def solo_phase(a, dev, steps, warmup):
    """1-GPU figure of the same step (rank 0, no communicator) in this run."""
    engine, sync, it = build(a, dev, 0, 1, NullComm())
    step = make_step(engine, sync, it)
    for _ in range(warmup):
        step()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    del engine, sync, it
    gc.collect()
    if dev.type == "cuda":
        torch.cuda.empty_cache()
    return a.batch * steps / el


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    gpus = a.gpus if a.gpus is not None else env_world
    rc = benchlib.relaunch(os.path.abspath(__file__), argv, gpus, a.profile, a.profile_dir, a.launch_timeout)
    if rc is not None:
        return rc
    if "WORLD_SIZE" in os.environ and a.gpus is not None and a.gpus != env_world:
        raise SystemExit(f"--gpus {a.gpus} but the launcher started WORLD_SIZE={env_world} ranks")
    launcher = "spawn" if is_spawned_child() else ("torchrun" if "TORCHELASTIC_RUN_ID" in os.environ or
                                                   "WORLD_SIZE" in os.environ else "single")
    torch_ref = None
    if a.torch_baseline > 0 and gpus == 1 and a.model == "VGG11":  # before this process touches the GPU
        torch_ref = benchlib.torch_eager_baseline(a.torch_baseline, min(a.warmup, 10), a.batch)
    ctx = init_env(device=a.device, comm=a.comm)
    dev = ctx.device
    torch.manual_seed(1)

    solo_img_s = None
    solo_steps = min(a.steps, 30) if a.solo_steps is None else a.solo_steps
    if ctx.world > 1 and solo_steps > 0:
        if ctx.rank == 0:
            solo_img_s = solo_phase(a, dev, solo_steps, min(a.warmup, 5))
        ctx.barrier()

    if a.ipc == "on" and ipc_possible(ctx, dev):
        store = ctx.store if ctx.store is not None else torch.distributed.distributed_c10d._get_default_store()
        ctx.comm = IpcComm(ctx.comm, store, dev)
    engine, sync, batches = build_parts(a, dev, ctx.rank, ctx.world, ctx.comm)
    sync, tune_report = tune_comm(a, engine, sync, ctx, dev, batches)
    it = batches()
    graphed = (GraphedStep(engine, sync, fallback=a.graph == "auto")
               if a.graph != "off" and ctx.world == 1 and not sync.active and dev.type == "cuda" else None)
    el = benchlib.timed_steps(make_step(engine, sync, it, graphed), a.steps, a.warmup, ctx, dev)
    engine.check_signals()
    loss = float(engine.loss.item())
    ms = el / a.steps * 1e3
    img_s = a.batch * ctx.world * a.steps / el

    diag = None
    live = [] if isinstance(ctx.comm, IpcComm) else None
    if a.diag_steps > 0 and dev.type == "cuda":
        probe = EventProbe(dev)
        sync.probe = probe
        step = make_step(engine, sync, it, probe=probe)
        samples = []
        for _ in range(a.diag_steps):
            probe.reset()
            probe.mark("start")
            step()
            samples.append(probe.times())
            if live is not None:  # (after the step's own timing: the check re-reduces the arena)
                ipc_live_checks(ctx.comm, engine, live)
        sync.probe = None
        sync.__dict__.pop("finish", None)  # drop make_step's probe wrapper
        engine.check_signals()  # (the diagnostic steps' bounded waits too)
        diag = step_comm_report(samples, len(sync.buckets))
        diag["exposed_comm_ms"] = ctx.all_max(diag["exposed_comm_ms"] or 0.0)
    benchlib.device_barrier(ctx, dev)
    pdiff = benchlib.replicas_max_diff(ctx.comm, engine.params.flat)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    cw = benchlib.comm_world(ctx.comm)
    checksum = float(engine.params.flat.double().sum().item())  # cross-mode oracle

    if ctx.rank == 0:
        base = BASELINE_IMG_S.get(ctx.world)
        per_gpu = img_s / ctx.world
        rec = {
            "metric": BASELINE_METRIC,
            "value": round(img_s, 1),
            "unit": "images/sec",
            "n_gpus": ctx.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(img_s / base, 2) if base else None,
            "dtype": "bf16" if a.impl == "bf16" else "fp32",
            "conv_impl": a.impl,
            "hip_graph": graphed is not None and graphed.graph is not None,
            "data": "synthetic (CIFAR-10-shaped uint8 on device, random-crop/flip/normalize each step)",
            "config": {"model": a.model, "global_batch": a.batch * ctx.world, "seq_len": None, "image_size": 32,
                       "parallelism": f"dp{ctx.world}",
                       # one rank without a communicator runs no collective at all
                       "sync_mode": a.mode if sync.active else f"none (1 rank, no collectives; {a.mode} requested)",
                       "comm": ctx.comm.name,
                       "bucket_mb": [round(4 * b.numel / 2 ** 20, 3) for b in sync.buckets] if sync.active else None,
                       "per_bucket_update": bool(sync.fuse_step), "comm_tune": tune_report,
                       "overlap": not a.no_overlap, "launcher": launcher,
                       "optimizer": "SGD(lr=0.1, momentum=0.9, wd=1e-4)"},
            "per_gpu_img_s": round(per_gpu, 1),
            "solo_img_s": round(solo_img_s, 1) if solo_img_s else None,
            "scaling_efficiency": round(per_gpu / solo_img_s, 4) if solo_img_s else None,
            "rccl_world": cw,
            # seconds this rank spent creating the main RCCL communicator (ncclCommInitRankConfig)
            "rccl_init_s": round(ctx.comm.init_s, 3) if getattr(ctx.comm, "init_s", None) is not None else None,
            "ipc_allreduce_ops": getattr(ctx.comm, "ipc_ops", None),
            # peer-memory collectives by kind, and collectives the IPC communicator handed to the
            # communicator it wraps (0 with --comm ipc: no tensor byte through gloo / the host)
            "ipc_ops_by_kind": dict(ctx.comm.ops) if hasattr(ctx.comm, "ops") else None,
            "ipc_inner_tensor_ops": getattr(ctx.comm, "inner_tensor_ops", None),
            # store-side agreement checks of the peer all-reduce on the live gradient arena, one per
            # diagnostic step (None: no peer-memory communicator)
            "ipc_live_check": (None if live is None else
                               {"checks": len(live), "ok": all(c["ok"] for c in live),
                                "max_rel_err": max((c["rel_err"] for c in live), default=None)}),
            "replicas_identical": pdiff == 0.0,
            "replica_param_max_diff": pdiff,
            "comm_diag": diag,
            # same-run stock-torch comparison (only with --torch-baseline; None otherwise)
            "torch_eager_fp32_img_s": round(torch_ref["img_per_s"], 1) if torch_ref else None,
            "vs_torch_eager_fp32": round(img_s / torch_ref["img_per_s"], 3) if torch_ref else None,
            "final_loss": round(loss, 4),
            "param_checksum": checksum,
        }
        print(json.dumps(rec), flush=True)
    ctx.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
