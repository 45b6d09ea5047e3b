"""Cost of cross-stream dependency events on MI355X (one GPU).

    python tools/event_overhead.py [--n 200]

Chains of small kernels (one 4 MiB in-place add each) on one stream, timed with host clocks
around a synchronize:
  plain          no events
  rec:<kind>     an event recorded between every two kernels
  ping:<kind>    two streams alternate kernels, each waiting on the other's event
kind: torch (torch.cuda.Event = system-scope release), device (hipEventReleaseToDevice),
nofence (hipEventDisableSystemFence).  Also a 'reuse' pass: after each event, a kernel re-reads a
64 MiB L2/MALL-resident tensor, to expose the cost of the cache writeback/invalidate.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_amd import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    a = ap.parse_args()
    C = _ext.require()
    dev = torch.device("cuda", 0)
    x = torch.zeros(1 << 20, device=dev)
    big = torch.ones(16 << 20, device=dev)
    out = torch.zeros(1, device=dev)  # noqa
    s0 = torch.cuda.current_stream(dev)
    s1 = torch.cuda.Stream(dev)
    flags = {"device": C.EVENT_DISABLE_TIMING | C.EVENT_RELEASE_TO_DEVICE,
             "nofence": C.EVENT_DISABLE_TIMING | C.EVENT_DISABLE_SYSTEM_FENCE}

    def mk(kind):
        if kind == "torch":
            return [torch.cuda.Event() for _ in range(2)]
        return [C.DevEvent(flags[kind]) for _ in range(2)]

    def rec(ev, s):
        if isinstance(ev, torch.cuda.Event):
            ev.record(s)
        else:
            ev.record(s.cuda_stream)

    def wait(ev, s):
        if isinstance(ev, torch.cuda.Event):
            s.wait_event(ev)
        else:
            ev.wait(s.cuda_stream)

    def timeit(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best * 1e6 / a.n  # us per kernel

    res = {}
    res["plain"] = timeit(lambda: [x.add_(1.0) for _ in range(a.n)])

    def reuse_plain():
        for _ in range(a.n):
            torch.sum(big, dim=0, out=out[0])
    res["reuse_plain"] = timeit(reuse_plain)
    for kind in ("torch", "device", "nofence"):
        evs = mk(kind)

        def recs():
            for _ in range(a.n):
                x.add_(1.0)
                rec(evs[0], s0)
        res[f"rec:{kind}"] = timeit(recs)

        def reuse():
            for _ in range(a.n):
                torch.sum(big, dim=0, out=out[0])
                rec(evs[0], s0)
        res[f"reuse:{kind}"] = timeit(reuse)

        def ping():
            for i in range(a.n):
                s, o = (s0, s1) if i % 2 == 0 else (s1, s0)
                with torch.cuda.stream(s):
                    x.add_(1.0)
                rec(evs[i % 2], s)
                wait(evs[i % 2], o)
            s0.wait_stream(s1)
        res[f"ping:{kind}"] = timeit(ping)
    print(json.dumps({k: round(v, 2) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
