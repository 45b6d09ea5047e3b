"""Host enqueue time of the headline step vs its device time: is the step launch-bound?

    python tools/host_enqueue.py [bench.py args]      (DPA_FORCE_COMM=1: through a 1-rank RCCL comm)

Runs 20 warmup steps, then 50 steps twice: once timing only the host side of each ``step()`` call
(no synchronisation inside the window), once timing the whole window with a final synchronize.  A
host time per step close to the device time per step means the GPU waits for launches.
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from distributed_pytorch_amd.parallel import init_env  # noqa: E402


def main():
    a = bench.parse(sys.argv[1:])
    ctx = init_env(device=a.device, comm=a.comm)
    dev = ctx.device
    engine, sync, it = bench.build(a, dev, ctx.rank, ctx.world, ctx.comm)
    step = bench.make_step(engine, sync, it)
    for _ in range(20):
        step()
    torch.cuda.synchronize(dev)
    n = 50
    host = []
    t0 = time.perf_counter()
    for _ in range(n):
        h = time.perf_counter()
        step()
        host.append(time.perf_counter() - h)
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    t_all = time.perf_counter() - t0
    host.sort()
    print(json.dumps({"comm": ctx.comm.name, "sync_active": sync.active,
                      "host_ms_per_step_median": round(host[n // 2] * 1e3, 4),
                      "host_ms_per_step_max": round(host[-1] * 1e3, 4),
                      "issue_ms_per_step": round(t_issue / n * 1e3, 4),
                      "device_ms_per_step": round(t_all / n * 1e3, 4)}), flush=True)
    ctx.shutdown()


if __name__ == "__main__":
    main()
