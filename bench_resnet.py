"""Stress benchmark: ResNet-50, ImageNet-shaped, bf16 MFMA compute, DDP (BASELINE.json config 5).

New scope (the reference has only VGG-11).  Per-GPU batch is fixed (weak scaling); synthetic
ImageNet-shaped data (224x224x3 NHWC, 1000 classes) resident on the device; random init.
Every timed step: forward, loss, backward with bucketed RCCL all-reduce issued from gradient
hooks (parallel/ddp.py), fused SGD(0.1, 0.9, wd 1e-4).

    python bench_resnet.py [--gpus N] [--batch 128] [--steps 20] [--warmup 5] [--impl bf16|x3] [--profile]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench_resnet.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_pytorch_amd.models.resnet import resnet50  # noqa: E402
from distributed_pytorch_amd.parallel import init_env  # noqa: E402
from distributed_pytorch_amd.parallel.ddp import DistributedDataParallel, FlatSGD  # noqa: E402
from distributed_pytorch_amd.utils import benchlib  # noqa: E402


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE, else 1); without a "
                    "launcher environment N>1 starts N local ranks (parallel/spawn.py)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128, help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--impl", default="bf16", choices=["bf16", "x3"])
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    ap.add_argument("--comm", default="rccl", choices=["rccl", "ipc", "torch", "gloo"])
    ap.add_argument("--autotune", action="store_true",
                    help="time every conv kernel config during warmup and save tuning/generic_mi355x.json")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="1 GPU: capture the whole training step (forward, backward through autograd, fused SGD) "
                         "as one HIP graph after the warmup and replay it (removes the host/autograd gaps "
                         "between kernels: +2.3 %% at batch 128, docs/PERF_NOTES.md).  auto = on for one rank "
                         "(the multi-rank step issues its collectives from autograd hooks and stays eager)")
    ap.add_argument("--profile", action="store_true", help="re-run under rocprofv3 --kernel-trace --stats")
    ap.add_argument("--profile-dir", default="gpurun_out/prof_resnet")
    ap.add_argument("--launch-timeout", type=float, default=1800.0)
    a = ap.parse_args(argv)
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    rc = benchlib.relaunch(os.path.abspath(__file__), argv, a.gpus if a.gpus is not None else env_world, a.profile,
                           a.profile_dir, a.launch_timeout)
    if rc is not None:
        return rc
    ctx = init_env(comm=a.comm)
    dev = ctx.device
    torch.manual_seed(1)
    model = resnet50(1000, a.impl).to(dev)
    ddp = DistributedDataParallel(model, ctx.comm, bucket_mb=a.bucket_mb)
    opt = FlatSGD(ddp, lr=0.1, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator(device=dev).manual_seed(100 + ctx.rank)
    x = torch.randn(a.batch, a.image, a.image, 3, device=dev, generator=g)
    t = torch.randint(0, 1000, (a.batch,), device=dev, generator=g)

    one = torch.ones((), device=dev)  # the loss-gradient seed, allocated once (no fill kernel per step)

    def step():
        opt.zero_grad()
        loss = ddp(x, t)  # fused GAP + Linear + softmax-CE head (ops/functional.HeadCE)
        loss.backward(one)
        opt.step(ddp.finish())
        return loss

    if a.autotune:
        from distributed_pytorch_amd.ops import functional as Fn

        Fn.set_autotune(True)
        step()  # tunes every conv call of the step (outside the timed region)
        Fn.set_autotune(False)
        if ctx.rank == 0:
            Fn.save_tuning_table()
    last = {}

    def timed_step():
        last["loss"] = step()

    graphed = False
    if a.graph in ("on", "auto") and ctx.world == 1 and dev.type == "cuda" and not a.autotune:
        # torch.cuda.graph recipe: eager warmup on a side stream, then capture one whole step.  The
        # replays run the identical kernels on the same static input / parameter / gradient
        # buffers; only the Python host work (autograd graph walk, launches) disappears.
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(max(3, a.warmup)):
                step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(graph):
                static_loss = step()
            graphed = True
        except RuntimeError as err:  # capture refused: time the eager step, and say so
            if a.graph == "on":
                raise
            print(f"[bench_resnet] stream capture failed ({err}); timing the eager step", file=sys.stderr, flush=True)
            torch.cuda.synchronize(dev)

        if graphed:
            def timed_step():
                graph.replay()
                last["loss"] = static_loss

    el = benchlib.timed_steps(timed_step, a.steps, a.warmup, ctx, dev)  # max over ranks
    loss = last["loss"]
    pdiff = benchlib.replicas_max_diff(ctx.comm, ddp.flat_params)
    img_s = a.batch * ctx.world * a.steps / el
    if ctx.rank == 0:
        print(json.dumps({
            "metric": f"images/sec ResNet-50 ImageNet-shaped training (batch {a.batch}/GPU)",
            "value": round(img_s, 1), "unit": "images/sec", "n_gpus": ctx.world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if a.impl == "bf16" else "fp32",
            "data": "synthetic (ImageNet-shaped 224x224x3 on device, random labels)",
            "config": {"model": "resnet50", "global_batch": a.batch * ctx.world, "seq_len": None,
                       "image_size": a.image, "parallelism": f"dp{ctx.world}", "buckets": ddp.num_buckets(),
                       "hip_graph": graphed,
                       "comm": ctx.comm.name, "optimizer": "SGD(lr=0.1, momentum=0.9, wd=1e-4)"},
            "rccl_world": benchlib.comm_world(ctx.comm), "replicas_identical": pdiff == 0.0,
            "final_loss": round(float(loss.item()), 4),
        }), flush=True)
    ctx.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
