"""Headline benchmark: VGG-11 / CIFAR-10-shaped training throughput (images/sec, whole job).

BASELINE.json metric: "images/sec whole-node VGG-11 CIFAR-10 at 1/2/4/8 MI355X".  Config is the
reference's: VGG-11 (BN), batch 256 per rank (weak scaling), SGD(0.1, 0.9, wd 1e-4), fp32 compute
(the reference trains in fp32), synthetic CIFAR-shaped data on device, random init (seed 1).
Every timed step is a full training step: on-device augmentation of the batch, forward, loss,
backward, gradient synchronisation (DDP mode by default: bucketed RCCL all-reduce overlapped with
backward + BN-buffer broadcast), fused SGD update.

    python bench.py [--gpus 1] [--steps 50] [--warmup 10] [--mode ddp|allreduce|gather]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_pytorch_amd.data import DeviceLoader, ShardSampler, synthetic_cifar  # noqa: E402
from distributed_pytorch_amd.engine import VGGEngine  # noqa: E402
from distributed_pytorch_amd.graph_step import GraphedStep  # noqa: E402
from distributed_pytorch_amd.parallel import init_env, make_sync  # noqa: E402

BASELINE_METRIC = "images/sec whole-node VGG-11 CIFAR-10 at 1/2/4/8 MI355X; scaling efficiency"  # BASELINE.json
# BASELINE.md (reference harness measured on CPU — the only numbers the reference has)
BASELINE_IMG_S = {1: 397.8, 2: 601.8}
# stock PyTorch-ROCm eager fp32 on one MI355X (tools/torch_baseline.py, profiles/)
TORCH_EAGER_IMG_S_PER_GPU = 68699.5


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch (reference: 256 per node)")
    ap.add_argument("--mode", default="ddp", choices=["ddp", "allreduce", "gather", "zero1"])
    ap.add_argument("--model", default="VGG11")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "torch"])
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--graph", default="off", choices=["auto", "off", "on"],
                    help="single GPU: replay the captured step as a HIP graph (graph_step.py; auto = on with an "
                         "eager fallback).  Off by default: same throughput on MI355X (host enqueue 0.67 -> 0.27 "
                         "ms hides behind 1.7 ms of GPU work) and the graph executor reorders the two-stream "
                         "backward")
    ap.add_argument("--impl", default="x3", choices=["fp32", "x3", "bf16"],
                    help="conv kernels: x3 = fp32-grade results from bf16 matrix cores (3 bf16 planes per "
                         "operand, 6 plane products; default) | fp32 = fp32 MFMA | bf16 = mixed precision")
    a = ap.parse_args()

    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws != a.gpus:
        if a.gpus > 1 and ws == 1:
            raise SystemExit("for --gpus > 1 launch with torch.distributed.run (one rank per GPU)")
    ctx = init_env(device=a.device, comm=a.comm)
    dev = ctx.device
    torch.manual_seed(1)
    train = synthetic_cifar(50000, 0)
    sampler = ShardSampler(len(train), ctx.world, ctx.rank, shuffle=True, seed=0)
    loader = DeviceLoader(train, a.batch, dev, sampler=sampler, train=True, seed=7919 + ctx.rank, drop_last=True)
    engine = VGGEngine(a.model, dev, max_batch=a.batch, impl=a.impl)
    engine.init_parameters(seed=1)
    sync = make_sync(a.mode, engine, ctx.comm, bucket_mb=a.bucket_mb, overlap=not a.no_overlap)

    def batches():
        ep = 0
        while True:
            loader.set_epoch(ep)
            yield from loader  # drop_last: every step has the full per-GPU batch
            ep += 1

    it = batches()
    graphed = (GraphedStep(engine, sync, fallback=a.graph == "auto")
               if a.graph != "off" and ctx.world == 1 and not sync.active and dev.type == "cuda" else None)

    def step():
        x, t = next(it)
        if graphed is not None:
            graphed.run(x, t)
            return
        sync.begin_step()
        engine.forward_backward(x, t, grad_ready=sync.grad_ready, pre_forward=sync.pre_forward,
                                params_free=sync.params_free)
        sync.update(sync.finish())
        engine.finish_step()

    for _ in range(a.warmup):
        step()

    def barrier():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        ctx.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    barrier()
    el = time.perf_counter() - t0
    el = ctx.all_max(el)  # slowest rank
    loss = float(engine.loss.item())
    ms = el / a.steps * 1e3
    img_s = a.batch * ctx.world * a.steps / el
    if ctx.rank == 0:
        base = BASELINE_IMG_S.get(ctx.world)
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
                       "parallelism": f"dp{ctx.world}", "sync_mode": a.mode, "comm": ctx.comm.name,
                       "optimizer": "SGD(lr=0.1, momentum=0.9, wd=1e-4)"},
            "vs_torch_eager_fp32": round(img_s / (TORCH_EAGER_IMG_S_PER_GPU * ctx.world), 3),
            "final_loss": round(loss, 4),
        }
        print(json.dumps(rec), flush=True)
    ctx.shutdown()


if __name__ == "__main__":
    main()
