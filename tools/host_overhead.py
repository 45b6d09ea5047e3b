"""How long the host takes to ENQUEUE one VGG training step, against how long the GPU takes to run
it.  If the enqueue time approaches the GPU time the step is launch-bound (the GPU waits on
Python), which is what graph replay (``--graph``) removes.

    python tools/host_overhead.py [--impl x3] [--steps 20] [--graph]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_pytorch_amd.data import DeviceLoader, ShardSampler, synthetic_cifar  # noqa: E402
from distributed_pytorch_amd.engine import VGGEngine  # noqa: E402
from distributed_pytorch_amd.parallel import make_sync  # noqa: E402
from distributed_pytorch_amd.parallel.comm import NullComm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", default="x3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    train = synthetic_cifar(50000, 0)
    loader = DeviceLoader(train, a.batch, dev, sampler=ShardSampler(len(train), 1, 0, True, 0), train=True,
                          seed=7919, drop_last=True)
    eng = VGGEngine("VGG11", dev, max_batch=a.batch, impl=a.impl)
    eng.init_parameters(seed=1)
    sync = make_sync("ddp", eng, NullComm())
    it = iter(loader)

    def step():
        x, t = next(it)
        sync.begin_step()
        eng.forward_backward(x, t, grad_ready=sync.grad_ready, pre_forward=sync.pre_forward,
                             params_free=sync.params_free)
        sync.update(sync.finish())
        eng.finish_step()

    runner = step
    if a.graph:
        from distributed_pytorch_amd.train import GraphedStep

        gs = GraphedStep(eng, sync, loader)
        runner = gs.step
    for _ in range(5):
        runner()
    torch.cuda.synchronize()
    host = []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        runner()
        host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        runner()
    torch.cuda.synchronize()
    gpu = (time.perf_counter() - t0) / a.steps
    host.sort()
    print(json.dumps({"impl": a.impl, "graph": a.graph, "host_enqueue_ms_median": round(host[len(host) // 2] * 1e3, 3),
                      "host_enqueue_ms_min": round(host[0] * 1e3, 3), "step_ms": round(gpu * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
