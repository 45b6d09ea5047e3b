"""Measure what the gradient-sync machinery costs on ONE GPU (no peers): the same VGG step with
NullComm, with a side stream that only carries the region/wait fences, and with the native 1-rank
RCCL communicator (normal / high-priority comm stream, collectives issued or skipped).

    python tools/comm_overhead.py [--steps 30] [--mode ddp]
"""
import argparse
import contextlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_pytorch_amd import _ext  # noqa: E402
from distributed_pytorch_amd.engine import VGGEngine  # noqa: E402
from distributed_pytorch_amd.parallel import make_sync  # noqa: E402
from distributed_pytorch_amd.parallel.comm import Comm, NullComm, RcclComm  # noqa: E402


class FenceOnly(Comm):
    """Side stream + the same event fences, but no collectives."""
    name = "fence"

    def __init__(self, dev, prio):
        self.rank, self.world = 0, 1
        self.dev = dev
        self.s = torch.cuda.Stream(dev, priority=-1 if prio else 0)

    @contextlib.contextmanager
    def region(self):
        self.s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(self.s):
            yield

    def all_reduce(self, t, op="sum"):
        pass

    def broadcast(self, t, root=0):
        pass

    def gather(self, send, recv, root=0):
        if recv is not None:
            recv.view(-1)[: send.numel()].copy_(send.view(-1))

    def wait(self):
        torch.cuda.current_stream(self.dev).wait_stream(self.s)


class RcclSkip(RcclComm):
    name = "rccl_skip"

    def all_reduce(self, t, op="sum"):
        pass

    def broadcast(self, t, root=0):
        pass


def run(comm, mode, steps, warmup, batch):
    dev = torch.device("cuda", 0)
    e = VGGEngine("VGG11", dev, max_batch=batch, impl="x3")
    e.init_parameters(seed=1)
    sync = make_sync(mode, e, comm)
    x = torch.randn(batch, 32, 32, 4, device=dev)
    x[..., 3] = 0
    t = torch.randint(0, 10, (batch,), device=dev)

    def step():
        sync.begin_step()
        e.forward_backward(x, t, grad_ready=sync.grad_ready, pre_forward=sync.pre_forward,
                           params_free=sync.params_free)
        sync.update(sync.finish())
        e.finish_step()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--mode", default="ddp")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    C = _ext.require()
    variants = [
        ("null", lambda: NullComm()),
        ("fence", lambda: FenceOnly(dev, False)),
        ("fence_hiprio", lambda: FenceOnly(dev, True)),
        ("rccl_skip", lambda: RcclSkip(0, 1, dev, uid=C.rccl_unique_id())),
        ("rccl", lambda: RcclComm(0, 1, dev, uid=C.rccl_unique_id())),
    ]
    for name, mk in variants:
        comm = mk()
        ms = run(comm, a.mode, a.steps, a.warmup, a.batch)
        print(json.dumps({"variant": name, "mode": a.mode, "ms_per_step": round(ms, 4)}), flush=True)
        comm.close()


if __name__ == "__main__":
    main()
