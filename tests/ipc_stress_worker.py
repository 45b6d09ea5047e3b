"""One rank of the peer-memory all-reduce stress test (tests/test_multirank_gpu.py): the training
pattern -- a kernel on the compute stream rewrites the registered arena, the all-reduce runs on the
communicator's stream right behind it, the compute stream reads the result -- repeated with new data
every iteration, so a read of a peer's memory that returns an earlier iteration's bytes (a stale
cache line) shows up as a wrong sum.  Values are small integers: every sum is exact in fp32.
Prints one JSON line per rank (mismatching iterations and elements)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_amd.parallel import init_env  # noqa: E402


def main():
    os.environ.setdefault("DPA_IPC_BLOCKS", "16")
    ctx = init_env(comm="ipc")
    dev, W, r, c = ctx.device, ctx.world, ctx.rank, ctx.comm
    iters = int(os.environ.get("DPA_IPC_STRESS_ITERS", "200"))
    n = int(os.environ.get("DPA_IPC_STRESS_N", str(1 << 20)))
    arena = torch.zeros(n + 64, device=dev)
    c.register(arena)
    pattern = (torch.arange(n, device=dev) % 97).float()
    tri = W * (W + 1) / 2
    # DPA_IPC_STRESS_SYNC=1: the host waits for every iteration's check (no work in flight across
    # iterations); 0 (default): the counts stay on the device, iterations overlap as training steps do
    host_sync = os.environ.get("DPA_IPC_STRESS_SYNC", "0") == "1"
    bad = torch.zeros(2, dtype=torch.int64, device=dev)  # [iterations with a mismatch, elements]
    offs = [0, 4, 128]  # slices at several offsets of the registered region
    for it in range(iters):
        off = offs[it % len(offs)]
        t = arena[off:off + n - 256]
        p = pattern[: t.numel()]
        # new bytes written by a kernel on the compute stream right before the collective
        torch.add(p * float(r + 1), float(it % 251), out=t)
        with c.region():
            c.all_reduce(t)
        c.wait()
        exp = p * tri + float(W * (it % 251))
        ne = (t != exp).sum()
        bad[0] += (ne > 0).long()
        bad[1] += ne
        if host_sync:
            torch.cuda.synchronize(dev)
    bad_iters, bad_elems = (int(v) for v in bad.tolist())
    tmo = c.timed_out()
    print(json.dumps({"rank": r, "world": W, "iters": iters, "bad_iters": bad_iters, "bad_elems": bad_elems,
                      "timeout": tmo}), flush=True)
    ctx.shutdown()
    return 0 if bad_iters == 0 and not tmo else 1


if __name__ == "__main__":
    sys.exit(main())
