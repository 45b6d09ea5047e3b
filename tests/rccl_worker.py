"""One rank of the multi-GPU RCCL tests (tests/test_rccl_gpu.py), started as a plain child process
with the torchrun environment (parallel/spawn.py sets it).  Goes through the production bootstrap:
``init_env`` → native C++ TCP store → ncclUniqueId exchange → native RCCL communicator.

    python tests/rccl_worker.py MODE STEPS OUTDIR [--fault-rank R] [--fault-step S]

Writes OUTDIR/MODE_RANK.pt with the parameter arena, the BN buffers after the first eval
pre-forward, the per-step losses and the rank's input batches (rank 0 re-runs the step
single-process from them as the oracle).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_amd.engine import VGGEngine  # noqa: E402
from distributed_pytorch_amd.parallel import init_env, make_sync  # noqa: E402

N = 32


def batches(rank, steps):
    g = torch.Generator().manual_seed(1000 + rank)
    out = []
    for _ in range(steps):
        x = torch.zeros(N, 32, 32, 4)
        x[..., :3] = torch.randn(N, 32, 32, 3, generator=g)
        out.append((x, torch.randint(0, 10, (N,), generator=g)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode")
    ap.add_argument("steps", type=int)
    ap.add_argument("outdir")
    ap.add_argument("--fault-rank", type=int, default=-1)
    ap.add_argument("--fault-step", type=int, default=-1)
    ap.add_argument("--bucket-mb", type=float, default=None)
    a = ap.parse_args()
    ctx = init_env(device="cuda", comm="rccl")
    dev = ctx.device
    e = VGGEngine("VGG11", dev, max_batch=N, impl="x3", lr=0.01)
    e.init_parameters(seed=1 + ctx.rank)  # different init per rank: the start-up broadcast must unify them
    sync = make_sync(a.mode, e, ctx.comm, bucket_mb=a.bucket_mb)
    data = batches(ctx.rank, a.steps)
    losses = []
    for s, (x, t) in enumerate(data):
        if ctx.rank == a.fault_rank and s == a.fault_step:
            print(f"[rank {ctx.rank}] injected exit at step {s}", flush=True)
            os._exit(13)
        sync.begin_step()
        e.forward_backward(x.to(dev), t.to(dev), grad_ready=sync.grad_ready, pre_forward=sync.pre_forward,
                           params_free=sync.params_free)
        sync.update(sync.finish())
        e.finish_step()
        losses.append(float(e.loss.item()))
    if a.mode in ("ddp", "zero1"):
        wait = sync.pre_forward()  # the first eval forward broadcasts rank 0's buffers (DDP semantics)
        if wait is not None:
            wait()
    torch.cuda.synchronize(dev)
    ctx.comm.check()
    torch.save({"params": e.params.flat.cpu(), "buffers": e.buffers.flat.cpu(), "losses": losses,
                "world": ctx.world, "comm": ctx.comm.name, "rccl_world": ctx.comm.comm_count(),
                "data": data}, os.path.join(a.outdir, f"{a.mode}_{ctx.rank}.pt"))
    ctx.barrier()
    ctx.shutdown()


if __name__ == "__main__":
    main()
