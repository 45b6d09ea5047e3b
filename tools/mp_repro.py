"""Multi-process one-GPU reproducibility probe (VERDICT r5 "what's missing" #1).

Runs P processes on the same GPU at once; every process loops a producer -> consumer pattern with
a known answer for ``--seconds`` and counts, ON THE DEVICE (no host sync inside the loop), every
consumer that saw anything but the answer.  Patterns (``--mode``):

  fill     torch only: X.fill_(i), then count X != i (one stream; no framework kernel at all)
  conv0    the framework's first-layer conv on FIXED inputs, output compared with the first one
  conv0alt conv0 on an input alternately copied from two sources (a producer kernel right before)
  signal   producer on stream A (fill), kernel-start signal (set_signal) on A, stream B polls it
           (wait_signal) and checks X -- the engine's cross-stream hand-off, alone

    python tools/mp_repro.py --procs 4 --seconds 15 --mode fill,conv0,conv0alt,signal
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(mode: str, seconds: float, rank: int) -> dict:
    import torch

    sys.path.insert(0, ROOT)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    bad = torch.zeros((), dtype=torch.int64, device=dev)
    iters = 0
    g = torch.Generator(device="cpu").manual_seed(1234)
    if mode == "fill":
        X = torch.empty(1 << 18, device=dev)  # 1 MiB: stays in one XCD's L2 between iterations
        Y = torch.empty(1 << 22, device=dev)  # 16 MiB of other traffic
        t0 = time.time()
        while time.time() - t0 < seconds:
            for _ in range(50):
                v = float(iters % 1000)
                X.fill_(v)
                bad += (X != v).sum()
                Y.mul_(0.5)
                iters += 1
    elif mode in ("big", "bigev"):
        # torch only: a 64 MiB producer (the size of the first VGG layer's output at batch 256), a
        # second stream, events and small pinned-memory copies around it -- the host-visible
        # traffic of a training step -- then the check of every element
        X = torch.empty(1 << 24, device=dev)
        Y = torch.empty(1 << 22, device=dev)
        side = torch.cuda.Stream(dev)
        ev = torch.cuda.Event()
        host = torch.zeros(64, dtype=torch.int32).pin_memory()
        small = torch.zeros(64, dtype=torch.int32, device=dev)
        t0 = time.time()
        while time.time() - t0 < seconds:
            for _ in range(20):
                v = float(iters % 1000)
                X.fill_(v)
                if mode == "bigev":
                    ev.record()
                    side.wait_event(ev)
                    with torch.cuda.stream(side):
                        Y.mul_(0.5)
                    host.copy_(small, non_blocking=True)
                bad += (X != v).sum()
                iters += 1
            torch.cuda.synchronize()
    elif mode in ("conv0", "conv0alt"):
        from distributed_pytorch_amd import _ext

        K = _ext.require()
        N = 64
        xa = torch.zeros(N, 32, 32, 4)
        xa[..., :3] = torch.randn(N, 32, 32, 3, generator=g)
        xb = torch.zeros(N, 32, 32, 4)
        xb[..., :3] = torch.randn(N, 32, 32, 3, generator=g)
        w = torch.zeros(64, 3, 3, 4)
        w[..., :3] = torch.randn(64, 3, 3, 3, generator=g) * 0.2
        xa, xb, w = xa.to(dev), xb.to(dev), w.to(dev)
        x = xa.clone()
        z = torch.empty(N, 32, 32, 64, device=dev)
        K.conv0_fwd(xa, w, z)
        za = z.clone()
        K.conv0_fwd(xb, w, z)
        zb = z.clone()
        torch.cuda.synchronize()
        t0 = time.time()
        while time.time() - t0 < seconds:
            for _ in range(50):
                if mode == "conv0":
                    K.conv0_fwd(xa, w, z)
                    bad += (z != za).any()
                else:
                    src, ref = (xa, za) if iters % 2 == 0 else (xb, zb)
                    x.copy_(src)
                    K.conv0_fwd(x, w, z)
                    bad += (z != ref).any()
                iters += 1
    elif mode == "signal":
        from distributed_pytorch_amd import _ext

        K = _ext.require()
        X = torch.empty(1 << 18, device=dev)
        sig = torch.zeros(1, dtype=torch.int32, device=dev)
        tmo = torch.zeros(1, dtype=torch.int32, device=dev)
        sb = torch.cuda.Stream(dev)
        main = torch.cuda.current_stream(dev)
        ev = torch.cuda.Event()
        t0 = time.time()
        while time.time() - t0 < seconds:
            for _ in range(50):
                iters += 1
                v = float(iters % 1000)
                X.fill_(v)  # producer (main)
                K.set_signal(sig, iters)  # the next main-stream kernel signals at its start
                with torch.cuda.stream(sb):
                    K.wait_signal(sig, iters, 5_000_000, tmo)
                    bad += (X != v).sum()  # consumer (side stream)
                    ev.record(sb)
                main.wait_event(ev)  # the next producer waits for the consumer
        bad += tmo.long().sum() * 1_000_000
    else:
        raise SystemExit(f"unknown mode {mode}")
    torch.cuda.synchronize()
    return {"rank": rank, "mode": mode, "iters": iters, "bad": int(bad.item())}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--seconds", type=float, default=15.0)
    ap.add_argument("--mode", default="fill,conv0,conv0alt,signal")
    ap.add_argument("--child", default=None)
    ap.add_argument("--rank", type=int, default=0)
    a = ap.parse_args(argv)
    if a.child:
        print(json.dumps(child(a.child, a.seconds, a.rank)), flush=True)
        return 0
    rc = 0
    for mode in a.mode.split(","):
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", mode, "--seconds",
                                   str(a.seconds), "--rank", str(r)], stdout=subprocess.PIPE, env=env, text=True)
                 for r in range(a.procs)]
        rows = []
        for p in procs:
            out, _ = p.communicate(timeout=a.seconds + 240)
            if p.returncode != 0:
                rc = p.returncode
            rows += [json.loads(l) for l in out.splitlines() if l.startswith("{")]
        print(json.dumps({"mode": mode, "procs": a.procs, "rows": rows,
                          "bad_total": sum(r["bad"] for r in rows)}), flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
