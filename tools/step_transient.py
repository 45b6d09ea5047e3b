"""Per-step GPU time of the headline step from a cold start (tools for the driver-window gap).

    python tools/step_transient.py [--steps 60] [--warmup 5]

Builds the bench step exactly as bench.py does (1 rank), runs ``--warmup`` steps, synchronises,
then records a device event between consecutive steps and prints each step's ms plus the mean
over windows — the driver times steps warmup+1 .. warmup+20 of a fresh process.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from distributed_pytorch_amd.parallel import NullComm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--prewarm-ms", type=float, default=0.0,
                    help="diagnostic: busy the GPU with matmuls this long after the build, before the warmup "
                         "steps (does the transient follow the clock, or the process?)")
    ap.add_argument("--prewarm-kind", default="mfma", choices=["mfma", "mem"],
                    help="mfma: fp32 matmuls; mem: 1 GiB device copies (memory / fabric clocks)")
    ap.add_argument("--prelaunch", type=int, default=0,
                    help="diagnostic: this many tiny kernel launches before the warmup steps (launch-path state)")
    ap.add_argument("--lr", type=float, default=None, help="diagnostic: override the SGD learning rate (0: frozen)")
    a = ap.parse_args()
    args = bench.parse([])
    dev = torch.device("cuda", 0)
    t0 = time.perf_counter()
    engine, sync, it = bench.build(args, dev, 0, 1, NullComm())
    step = bench.make_step(engine, sync, it)
    if a.lr is not None:
        engine.lr = a.lr
    if a.prelaunch > 0:
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        for i in range(a.prelaunch):
            engine.K.set_signal(flag, i)
        torch.cuda.synchronize()
    if a.prewarm_ms > 0:
        big = a.prewarm_kind == "mem"
        x = torch.randn((1 << 28) if big else 4096 * 4096, device=dev)
        y = torch.empty_like(x) if big else None
        t1 = time.perf_counter()
        while (time.perf_counter() - t1) * 1e3 < a.prewarm_ms:
            for _ in range(8):
                if big:
                    y.copy_(x)
                else:
                    x = torch.tanh(x.view(4096, 4096) @ x.view(4096, 4096)).view(-1)
            torch.cuda.synchronize()
        del x, y
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    print(f"build+warmup {time.perf_counter() - t0:.2f} s", flush=True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    host = []
    ev[0].record()
    for i in range(a.steps):
        h = time.perf_counter()
        step()
        host.append((time.perf_counter() - h) * 1e3)
        ev[i + 1].record()
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(a.steps)]
    print("step gpu_ms host_ms")
    for i, (g, h) in enumerate(zip(ms, host)):
        print(f"{a.warmup + i + 1:4d} {g:7.4f} {h:7.3f}")
    for lo in range(0, a.steps, 10):
        w = ms[lo:lo + 10]
        print(f"steps {a.warmup + lo + 1}-{a.warmup + lo + len(w)}: mean {sum(w) / len(w):.4f} ms")


if __name__ == "__main__":
    main()
