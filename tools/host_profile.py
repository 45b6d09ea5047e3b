"""Host side of the bench step: enqueue time per step (host returns before the GPU finishes) and a
cProfile of the Python/C++ calls behind it, for the null communicator and a 1-rank RCCL one.

    python tools/host_profile.py [--comm null|rccl] [--steps 30] [--top 30]

A step whose enqueue time approaches its GPU time is launch-bound: the GPU idles between kernels.
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from distributed_pytorch_amd.parallel import NullComm, init_env  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--comm", default="null", choices=["null", "rccl"])
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    if a.comm == "rccl":
        os.environ["DPA_FORCE_COMM"] = "1"
        ctx = init_env(device="cuda", comm="rccl")
        comm, dev = ctx.comm, ctx.device
    else:
        dev, comm = torch.device("cuda", 0), NullComm()
    args = bench.parse([])
    engine, sync, it = bench.build(args, dev, 0, 1, comm)
    step = bench.make_step(engine, sync, it)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    host = []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    gpu = (time.perf_counter() - t0) / a.steps
    host.sort()
    print(json.dumps({"comm": a.comm, "host_enqueue_ms_median": round(host[len(host) // 2] * 1e3, 3),
                      "host_enqueue_ms_min": round(host[0] * 1e3, 3), "step_ms": round(gpu * 1e3, 3)}), flush=True)
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    pr.enable()
    for _ in range(a.steps):
        torch.cuda.synchronize()
        step()
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(a.top)
    print(s.getvalue())


if __name__ == "__main__":
    main()
