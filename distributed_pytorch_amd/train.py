"""Training / evaluation loop and the shared CLI behind every entry point.

Mirrors the reference's observable behaviour (main.py:19-66):
  * ``Epoch: {e}, Iteration: {a}-{b}, Average Loss: {x:.3f}`` every 20 iterations;
  * ``Avg Time for iteration 2-40: {t} seconds.`` then every 40 (iteration 0 excluded, first
    window ÷39);
  * ``Test set: Average loss: {:.4f}, Accuracy: {}/{} ({:.0f}%)`` over the full, unsharded test
    set on every rank;
  * every rank prints; seed 1 before model construction; sampler seed 0; batch 256 per rank;
    SGD(lr 0.1, momentum 0.9, wd 1e-4); 1 epoch.
Timing is device-accurate: the clock is read after a device synchronize at each window boundary
(the reference's ``loss.item()`` forced the same synchronisation every step).
Extra (new scope): images/sec, JSON metrics, per-rank checkpoints + resume, roctx tracing, RCCL
async-error polling.
"""
from __future__ import annotations

import argparse
import json
import os
import time
from typing import Optional

import torch

from .data import DeviceLoader, ShardSampler, get_datasets
from .engine import VGGEngine
from .graph_step import GraphedStep
from .parallel import DistContext, env_dict, init_cli, init_env, init_single, make_sync
from .utils import checkpoint
from .utils.profiling import enable_tracing, trace_range

BATCH_SIZE = 256  # main.py:18 ("batch for one node")


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _eager_step(engine: VGGEngine, sync, x: torch.Tensor, target: torch.Tensor):
    with trace_range("step"):
        sync.begin_step()
        with trace_range("fwd_bwd"):
            engine.forward_backward(x, target, grad_ready=sync.grad_ready, pre_forward=sync.pre_forward,
                                    params_free=sync.params_free)
        with trace_range("sync"):
            gscale = sync.finish()
        with trace_range("sgd"):
            sync.update(gscale)
        engine.finish_step()


def _fault_point(rank: int, it: int):
    """Fault injection: ``DPA_FAULT=rank:iter[:kind]`` makes that rank fail at that
    training iteration — ``exit`` (default: the process dies without cleanup, like a lost node),
    ``raise`` (a Python error) or ``hang`` (stops issuing collectives; peers must time out)."""
    spec = os.environ.get("DPA_FAULT")
    if not spec:
        return
    parts = spec.split(":")
    if int(parts[0]) != rank or int(parts[1]) != it:
        return
    kind = parts[2] if len(parts) > 2 else "exit"
    print(f"[rank {rank}] injected fault '{kind}' at iteration {it}", flush=True)
    if kind == "raise":
        raise RuntimeError(f"injected fault at iteration {it}")
    if kind == "hang":
        time.sleep(10 ** 6)
    os._exit(13)


def agreed_health_check(engine: VGGEngine, ctx: DistContext):
    """Before anything is saved: this rank's device error words (engine.check_signals: the per-step
    health snapshots, the wgrad-stream / BN-rendezvous timeouts, the fp16-pair overflow words) and
    its communicator's (ctx.comm.check: RCCL async errors, peer-collective timeouts), agreed over
    every rank -- a peer whose collectives timed out may have fed this rank a corrupted reduction
    while this rank's own words are clear, so every rank raises together or none does."""
    err = None
    try:
        engine.check_signals()
        ctx.comm.check()
    except RuntimeError as e:
        err = e
    if ctx.all_max(1.0 if err is not None else 0.0) > 0:
        raise err if err is not None else RuntimeError(
            f"[rank {ctx.rank}] a peer rank failed its health check; not saving results built on its collectives")


def train_model(engine: VGGEngine, loader: DeviceLoader, sync, epoch: int, ctx: DistContext, args,
                start_batch: int = 0, stats: Optional[dict] = None, budget: Optional[int] = None) -> Optional[int]:
    """One epoch (main.py:19-49).  ``budget`` caps the iterations run in this call (the remainder of
    ``--stop-after-iters``); returns the next batch index when the budget ran out mid-epoch, else None."""
    dev = engine.device
    engine.loss_accum.zero_()
    t_win, win_start = None, None
    n_iters = 0
    t_epoch0 = None
    stopped_at = None
    max_iters = getattr(args, "max_iters", None)
    ck_every = getattr(args, "checkpoint_every", 0) or 0
    graphed = GraphedStep(engine, sync) if getattr(args, "graph", False) and not sync.active and dev.type == "cuda" \
        else None
    for batch_idx, (x, target) in enumerate(loader.iterate(start_batch), start=start_batch):
        if graphed is not None:
            with trace_range("step_graph"):
                graphed.run(x, target)
        else:
            _eager_step(engine, sync, x, target)
        n_iters += 1
        _fault_point(ctx.rank, batch_idx)
        if batch_idx == start_batch:
            _sync(dev)
            t_win = time.perf_counter()
            t_epoch0 = t_win
            win_start = batch_idx
        if batch_idx % 20 == 19:
            running = float(engine.loss_accum.item())
            engine.loss_accum.zero_()
            print(f"Epoch: {epoch + 1}, Iteration: {batch_idx - 18}-{batch_idx + 1}, Average Loss: {running / 20:.3f}",
                  flush=True)
        if batch_idx % 40 == 39:
            _sync(dev)
            now = time.perf_counter()
            if batch_idx == 39:
                print(f"Avg Time for iteration {batch_idx - 37}-{batch_idx + 1}: {(now - t_win) / 39} seconds.",
                      flush=True)
            else:
                print(f"Avg Time for iteration {batch_idx - 38}-{batch_idx + 1}: {(now - t_win) / 40} seconds.",
                      flush=True)
            t_win = now
            ctx.comm.check()
        if ck_every and args.checkpoint_dir and (batch_idx + 1) % ck_every == 0:
            agreed_health_check(engine, ctx)  # never save weights built from a failed step, on any rank
            sync.prepare_checkpoint()
            checkpoint.save(args.checkpoint_dir, ctx.rank, engine, epoch, batch_idx + 1, args.sampler_seed, ctx.world,
                            sync.mode, ddp_prefix=sync.mode == "ddp")
        if max_iters and n_iters >= max_iters:
            break
        if budget is not None and n_iters >= budget and batch_idx + 1 < len(loader):
            stopped_at = batch_idx + 1
            break
    _sync(dev)
    if stats is not None and t_epoch0 is not None and n_iters > 1:
        el = time.perf_counter() - t_epoch0
        stats["iters_timed"] = n_iters - 1
        stats["sec_per_iter"] = el / (n_iters - 1)
        stats["images_per_sec_rank"] = loader.batch_size / stats["sec_per_iter"]
        stats["images_per_sec_total"] = stats["images_per_sec_rank"] * ctx.world
    if stats is not None:
        stats["iters_run"] = n_iters
    return stopped_at


def test_model(engine: VGGEngine, loader: DeviceLoader, sync=None):
    if sync is not None and sync.mode == "ddp":
        wait = sync.pre_forward()  # first eval forward under DDP still broadcasts rank 0's buffers
        if wait is not None:
            wait()
    engine.begin_eval()
    nb = 0
    for x, target in loader:
        engine.eval_batch(x, target)
        nb += 1
    acc = engine.eval_acc.cpu()
    test_loss = float(acc[0]) / max(nb, 1)
    correct = int(round(float(acc[1])))
    n = loader.dataset_len
    print("Test set: Average loss: {:.4f}, Accuracy: {}/{} ({:.0f}%)\n".format(test_loss, correct, n,
                                                                              100.0 * correct / n), flush=True)
    return test_loss, correct


def add_common_args(ap: argparse.ArgumentParser):
    g = ap.add_argument_group("framework options (defaults = reference values)")
    g.add_argument("--model", default="VGG11", choices=["VGG11", "VGG13", "VGG16", "VGG19"])
    g.add_argument("--epochs", type=int, default=1)
    g.add_argument("--batch-size", type=int, default=BATCH_SIZE, help="per-rank batch")
    g.add_argument("--lr", type=float, default=0.1)
    g.add_argument("--momentum", type=float, default=0.9)
    g.add_argument("--weight-decay", type=float, default=1e-4)
    g.add_argument("--seed", type=int, default=1)
    g.add_argument("--sampler-seed", type=int, default=0)
    g.add_argument("--data-root", default="./data")
    g.add_argument("--synthetic", action="store_true", help="synthetic CIFAR-shaped data (default if no dataset)")
    g.add_argument("--train-size", type=int, default=50000)
    g.add_argument("--test-size", type=int, default=10000)
    g.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    g.add_argument("--comm", default="rccl", choices=["rccl", "ipc", "torch", "gloo"])
    g.add_argument("--impl", default="h2", choices=["fp32", "x3", "h2", "bf16"],
                   help="GPU conv kernels: h2 (fp32-grade via fp16 pairs, default) | x3 (fp32-grade via "
                        "bf16 planes) | fp32 MFMA | bf16")
    g.add_argument("--bucket-mb", type=float, default=None)
    g.add_argument("--no-overlap", action="store_true", help="sync after backward (reference placement)")
    g.add_argument("--checkpoint-dir", default=None)
    g.add_argument("--checkpoint-every", type=int, default=0)
    g.add_argument("--resume", action="store_true")
    g.add_argument("--resume-reshard", action="store_true",
                   help="resume a checkpoint written with a different world size / sync mode: load weights and "
                        "optimizer state, restart its epoch at batch 0")
    g.add_argument("--max-iters", type=int, default=None, help="stop each epoch after this many iterations")
    g.add_argument("--stop-after-iters", type=int, default=None,
                   help="end the whole run after this many training iterations, mid-epoch if need be, writing a "
                        "resumable checkpoint (preemption drill for --resume)")
    g.add_argument("--no-eval", action="store_true")
    g.add_argument("--trace", action="store_true", help="emit roctx ranges (rocprofv3 --marker-trace)")
    g.add_argument("--profile", action="store_true",
                   help="re-run this command under rocprofv3 --kernel-trace --stats (prints the exact command; the "
                        "program follows '--' directly)")
    g.add_argument("--profile-dir", default="gpurun_out/prof_train")
    g.add_argument("--graph", action="store_true",
                   help="single rank: replay the training step as a captured HIP graph (graph_step.py)")
    g.add_argument("--json-metrics", default=None, help="append a JSON metrics line per epoch to this file")
    g.add_argument("--single-gpu-img-s", type=float, default=None,
                   help="1-GPU images/sec of the same config (e.g. bench.py --gpus 1): adds scaling_efficiency "
                        "to --json-metrics")
    g.add_argument("--port", type=int, default=6585)
    return ap


def resume(ctx: DistContext, engine: VGGEngine, mode: str, args, n_batches: int):
    """Load this rank's checkpoint (``--resume``) and check that every rank resumes from the same
    point; returns (start_epoch, start_batch).  Runs BEFORE the sync strategy's start-up broadcast,
    whose momentum broadcast depends on the (now agreed) step count."""
    if not (args.resume and args.checkpoint_dir):
        return 0, 0
    err, obj = None, None
    try:
        obj = checkpoint.load(args.checkpoint_dir, ctx.rank, engine, world=ctx.world, mode=mode,
                              reshard=getattr(args, "resume_reshard", False))
        point = checkpoint.resume_point(obj)
    except checkpoint.ResumeMismatch as e:
        err, point = e, (-1, -1, -1, -1)
    # every rank must resume from the same point (a collective: fails on all ranks, not one)
    checkpoint.agree(ctx.comm, point, ctx.device)
    if err is not None:
        raise err
    if obj is None:
        return 0, 0
    start_epoch, start_batch = obj["epoch"], obj["batch_idx"]
    if start_batch >= n_batches:
        start_epoch, start_batch = start_epoch + 1, 0
    return start_epoch, start_batch


def run(ctx: DistContext, mode: str, args):
    if args.trace:
        enable_tracing(True)
    torch.manual_seed(args.seed)  # main.py:70 — identical init on all ranks (plus a rank-0 broadcast)
    train_set, test_set = get_datasets(args.data_root, args.synthetic, args.train_size, args.test_size)
    sampler = ShardSampler(len(train_set), num_replicas=ctx.world, rank=ctx.rank, shuffle=True,
                           seed=args.sampler_seed, drop_last=False)
    train_loader = DeviceLoader(train_set, args.batch_size, ctx.device, sampler=sampler, train=True,
                                seed=args.seed * 7919 + ctx.rank)
    test_loader = DeviceLoader(test_set, args.batch_size, ctx.device, sampler=None, train=False)
    engine = VGGEngine(args.model, ctx.device, max_batch=args.batch_size, lr=args.lr, momentum=args.momentum,
                       weight_decay=args.weight_decay, impl=args.impl)
    engine.init_parameters(seed=args.seed)
    start_epoch, start_batch = resume(ctx, engine, mode, args, len(train_loader))
    sync = make_sync(mode, engine, ctx.comm, bucket_mb=args.bucket_mb, overlap=not args.no_overlap)
    budget = getattr(args, "stop_after_iters", None)
    for epoch in range(start_epoch, args.epochs):
        train_loader.set_epoch(epoch)
        stats = {}
        stopped = train_model(engine, train_loader, sync, epoch, ctx, args, start_batch=start_batch, stats=stats,
                              budget=budget)
        start_batch = 0
        agreed_health_check(engine, ctx)  # the epoch's waits, collectives and splits were all valid
        if budget is not None:
            budget -= stats.get("iters_run", 0)
        if stopped is not None:  # preempted mid-epoch: checkpoint the position, no eval
            if args.checkpoint_dir:
                sync.prepare_checkpoint()
                checkpoint.save(args.checkpoint_dir, ctx.rank, engine, epoch, stopped, args.sampler_seed, ctx.world,
                                mode, ddp_prefix=mode == "ddp")
            break
        if args.checkpoint_dir:
            sync.prepare_checkpoint()
            checkpoint.save(args.checkpoint_dir, ctx.rank, engine, epoch + 1, 0, args.sampler_seed, ctx.world, mode,
                            ddp_prefix=mode == "ddp")
        res = None
        if not args.no_eval:
            res = test_model(engine, test_loader, sync)
        if args.json_metrics and ctx.rank == 0:
            rec = dict(stats, epoch=epoch + 1, mode=mode, world=ctx.world, model=args.model,
                       batch_per_rank=args.batch_size, comm=ctx.comm.name)
            base = getattr(args, "single_gpu_img_s", None)
            if base and "images_per_sec_rank" in stats:
                # weak scaling: per-rank throughput relative to one GPU running alone
                rec["scaling_efficiency"] = stats["images_per_sec_rank"] / base
            if res:
                rec["test_loss"], rec["test_correct"] = res
            with open(args.json_metrics, "a") as f:
                f.write(json.dumps(rec) + "\n")
        if budget is not None and budget <= 0:
            break
    ctx.shutdown()


def _maybe_profile(args, argv) -> Optional[int]:
    """``--profile``: run this same command as a child under rocprofv3 (utils/benchlib.relaunch);
    this process touches no GPU and exits with the child's code."""
    if not getattr(args, "profile", False):
        return None
    import sys

    from .utils import benchlib

    argv = sys.argv[1:] if argv is None else list(argv)
    return benchlib.relaunch(os.path.abspath(sys.argv[0]), argv, 1, True, args.profile_dir, 0)


def main_cli(mode: str, argv=None):
    """``python main_{gather,all_reduce,part3}.py --master-ip IP --num-nodes N --rank R``"""
    ap = argparse.ArgumentParser(prog="Input arguments", description="gather ip, nunber of workers, rank")
    ap.add_argument("--master-ip", required=True)
    ap.add_argument("--num-nodes", required=True, type=int)
    ap.add_argument("--rank", required=True, type=int)
    add_common_args(ap)
    args = ap.parse_args(argv)
    rc = _maybe_profile(args, argv)
    if rc is not None:
        raise SystemExit(rc)
    ctx = init_cli(args.master_ip, args.num_nodes, args.rank, port=args.port, device=args.device, comm=args.comm)
    run(ctx, mode, args)


def main_env(mode: str = "ddp", argv=None):
    """``torchrun ... main_ddp.py`` (env:// rendezvous)."""
    ap = argparse.ArgumentParser(prog="Input arguments", description="gather ip, nunber of workers, rank")
    add_common_args(ap)
    args = ap.parse_args(argv)
    rc = _maybe_profile(args, argv)
    if rc is not None:
        raise SystemExit(rc)
    print(f"[{os.getpid()}] Initializing process group with: {env_dict()}", flush=True)
    ctx = init_env(device=args.device, comm=args.comm)
    run(ctx, mode, args)


def main_single(argv=None):
    """``python main.py`` — single process, no distribution (main.py:69-108)."""
    ap = argparse.ArgumentParser(prog="main.py")
    add_common_args(ap)
    args = ap.parse_args(argv)
    rc = _maybe_profile(args, argv)
    if rc is not None:
        raise SystemExit(rc)
    ctx = init_single(args.device)
    run(ctx, "allreduce", args)
