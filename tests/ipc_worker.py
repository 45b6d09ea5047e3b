"""One rank of the peer-memory all-reduce test (tests/test_multirank_gpu.py): ranks share the GPU
(parallel/spawn.py starts them; gloo carries the rendezvous), map each other's arenas through HIP
IPC and all-reduce slices of them with the native kernel.  Every rank regenerates every rank's data
from its seed and checks the result BITWISE against the rank-order fp32 sum.  Prints one JSON line
(rank 0)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_amd.parallel import init_env  # noqa: E402
from distributed_pytorch_amd.parallel.ipc import IpcComm  # noqa: E402


def main():
    ctx = init_env(comm="gloo")
    dev = ctx.device
    W, r = ctx.world, ctx.rank
    store = torch.distributed.distributed_c10d._get_default_store()
    c = IpcComm(ctx.comm, store, dev, blocks=int(os.environ.get("DPA_IPC_BLOCKS", "16")), timeout_s=30.0,
                stage_floats=int(os.environ.get("DPA_IPC_TEST_STAGE", str(1 << 22))))
    N = 1 << 21
    data = [torch.randn(N, generator=torch.Generator().manual_seed(100 + q)) for q in range(W)]
    arena = data[r].to(dev)
    c.register(arena)
    cases = [(0, N), (4, 1001), (1024, 3), (8, 4 * 777 + 2), (N - 4096, 4096)]
    ok = True
    for off, n in cases:
        exp = data[0][off:off + n].clone()
        for q in range(1, W):
            exp += data[q][off:off + n]
        before = arena.clone()
        with c.region():
            c.all_reduce(arena[off:off + n])
        c.wait()
        torch.cuda.synchronize(dev)
        got = arena[off:off + n].cpu()
        same = torch.equal(got, exp)
        untouched = torch.equal(torch.cat([arena[:off], arena[off + n:]]).cpu(),
                                torch.cat([before[:off], before[off + n:]]).cpu())
        ok = ok and same and untouched
        # restore this rank's own data for the next case (all ranks, then a barrier)
        arena.copy_(data[r].to(dev))
        torch.cuda.synchronize(dev)
        ctx.barrier()
    tmo = c._c.take_timeout()
    # timing: 10 MB all-reduces back to back (ranks share one GPU here: not a fabric number)
    t = arena[: (10 << 20) // 4]
    for _ in range(3):
        with c.region():
            c.all_reduce(t)
    c.wait()
    torch.cuda.synchronize(dev)
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(20):
        with c.region():
            c.all_reduce(t)
    c.wait()
    torch.cuda.synchronize(dev)
    el = ctx.all_max(time.perf_counter() - t0) / 20
    tmo = tmo or c._c.take_timeout()
    if r == 0:
        print(json.dumps({"world": W, "bitwise_ok": ok, "timeout": tmo, "ipc_ops": c.ipc_ops,
                          "ms_per_10MB_allreduce": round(el * 1e3, 4)}), flush=True)
    ctx.shutdown()
    return 0 if ok and not tmo else 1


if __name__ == "__main__":
    sys.exit(main())
