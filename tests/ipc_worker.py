"""One rank of the peer-memory collectives test (tests/test_multirank_gpu.py): ranks share the GPU
(torchrun starts them; the native store carries the rendezvous -- no torch.distributed group, no
gloo), map each other's memory through HIP IPC and run every collective of parallel/ipc.py on the
native kernels, through both input paths (registered memory read in place, and bounced through the
inbox).  Every rank regenerates every rank's data from its seed and checks each result BITWISE
against the rank-order fp32 reduction / the exact copy.  Prints one JSON line (rank 0)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_amd.parallel import init_env  # noqa: E402
from distributed_pytorch_amd.parallel.ipc import IpcComm  # noqa: E402


def rank_data(q, n, dtype=torch.float32):
    g = torch.Generator().manual_seed(100 + q)
    if dtype == torch.int64:
        return torch.randint(-2 ** 40, 2 ** 40, (n,), generator=g, dtype=torch.int64)
    return torch.randn(n, generator=g)


def main():
    os.environ.setdefault("DPA_IPC_BLOCKS", "16")
    ctx = init_env(comm="ipc")
    dev = ctx.device
    W, r = ctx.world, ctx.rank
    c = ctx.comm
    assert isinstance(c, IpcComm) and c.inner is None, type(c)
    stage = int(os.environ.get("DPA_IPC_TEST_STAGE", "0"))
    inbox = int(os.environ.get("DPA_IPC_TEST_INBOX", "0"))
    if stage or inbox:  # a second communicator with small buffers: every collective runs in pieces
        c = IpcComm(None, ctx.store, dev, rank=r, world=W, stage_words=stage or (1 << 22),
                    inbox_words=inbox or (1 << 22), timeout_s=30.0)
    results = {}

    def run(fn):
        with c.region():
            fn()
        c.wait()
        torch.cuda.synchronize(dev)

    def check(name, ok):
        results[name] = results.get(name, True) and bool(ok)

    N = 1 << 21
    data = [rank_data(q, N) for q in range(W)]
    arena = data[r].to(dev)
    c.register(arena)
    # 1. registered all-reduce (sum), slices with odd tails, nothing outside the slice touched
    for off, n in [(0, N), (4, 1001), (1024, 3), (8, 4 * 777 + 2), (N - 4096, 4096)]:
        exp = data[0][off:off + n].clone()
        for q in range(1, W):
            exp += data[q][off:off + n]
        before = arena.clone()
        run(lambda: c.all_reduce(arena[off:off + n]))
        check("all_reduce_registered", torch.equal(arena[off:off + n].cpu(), exp))
        check("all_reduce_untouched", torch.equal(torch.cat([arena[:off], arena[off + n:]]).cpu(),
                                                  torch.cat([before[:off], before[off + n:]]).cpu()))
        arena.copy_(data[r].to(dev))
        torch.cuda.synchronize(dev)
        c.barrier()
    # 2. bounced all-reduce: sum / max / min, odd length, an unaligned start
    for op, fn in (("sum", None), ("max", torch.maximum), ("min", torch.minimum)):
        n = 300_001
        exp = data[0][:n].clone()
        for q in range(1, W):
            exp = exp + data[q][:n] if fn is None else fn(exp, data[q][:n])
        buf = torch.empty(n + 1, device=dev)
        t = buf[1:]
        t.copy_(data[r][:n].to(dev))
        run(lambda: c.all_reduce(t, op))
        check(f"all_reduce_bounced_{op}", torch.equal(t.cpu(), exp))
    # 3. broadcast: registered and bounced, roots 0 and W-1, fp32 and int64
    for root in sorted({0, W - 1}):
        off, n = 12, 100_003
        arena.copy_(data[r].to(dev))
        run(lambda: c.broadcast(arena[off:off + n], root))
        check("broadcast_registered", torch.equal(arena[off:off + n].cpu(), data[root][off:off + n]))
        check("broadcast_untouched", torch.equal(arena[:off].cpu(), data[r][:off]))
        ti = rank_data(r, 5001, torch.int64).to(dev)
        run(lambda: c.broadcast(ti, root))
        check("broadcast_bounced_int64", torch.equal(ti.cpu(), rank_data(root, 5001, torch.int64)))
    # 4. gather: rank 0 receives every rank's slice (registered and bounced)
    arena.copy_(data[r].to(dev))
    n = 65_537
    recv = torch.full((W * n,), float("nan"), device=dev) if r == 0 else None
    run(lambda: c.gather(arena[4:4 + n], recv, 0))
    if r == 0:
        check("gather_registered", torch.equal(recv.cpu(), torch.cat([d[4:4 + n] for d in data])))
    priv = data[r][:n].to(dev)
    recv2 = torch.zeros(W * n, device=dev) if r == W - 1 else None
    run(lambda: c.gather(priv, recv2, W - 1))
    if r == W - 1:
        check("gather_bounced", torch.equal(recv2.cpu(), torch.cat([d[:n] for d in data])))
    # 5. reduce-scatter in place (ZeRO-1's form: the rank's own segment receives the sum) + bounced
    seg = 4 * 10_007
    exp_seg = data[0][r * seg:(r + 1) * seg].clone()
    for q in range(1, W):
        exp_seg += data[q][r * seg:(r + 1) * seg]
    arena.copy_(data[r].to(dev))
    run(lambda: c.reduce_scatter(arena[:W * seg], arena[r * seg:(r + 1) * seg]))
    check("reduce_scatter_registered", torch.equal(arena[r * seg:(r + 1) * seg].cpu(), exp_seg))
    src = data[r][:W * seg].to(dev)
    out = torch.empty(seg, device=dev)
    run(lambda: c.reduce_scatter(src, out))
    check("reduce_scatter_bounced", torch.equal(out.cpu(), exp_seg))
    # 6. all-gather in place (ZeRO-1's parameter form) + bounced
    arena.copy_(data[r].to(dev))
    run(lambda: c.all_gather(arena[r * seg:(r + 1) * seg], arena[:W * seg]))
    exp_ag = torch.cat([data[q][q * seg:(q + 1) * seg] for q in range(W)])
    check("all_gather_registered", torch.equal(arena[:W * seg].cpu(), exp_ag))
    piece = data[r][:seg + 3].to(dev)
    outg = torch.empty(W * (seg + 3), device=dev)
    run(lambda: c.all_gather(piece, outg))
    check("all_gather_bounced", torch.equal(outg.cpu(), torch.cat([data[q][:seg + 3] for q in range(W)])))
    c.barrier()
    tmo = c.timed_out()
    # timing: 10 MB registered all-reduces back to back (ranks share one GPU here: not a fabric number)
    arena.copy_(data[r].to(dev))
    t = arena[: (10 << 20) // 4]
    for _ in range(3):
        run(lambda: c.all_reduce(t))
    c.barrier()
    t0 = time.perf_counter()
    with c.region():
        for _ in range(20):
            c.all_reduce(t)
    c.wait()
    torch.cuda.synchronize(dev)
    el = ctx.all_max(time.perf_counter() - t0) / 20
    tmo = tmo or c.timed_out()
    ok = all(results.values())
    if r == 0:
        print(json.dumps({"world": W, "bitwise_ok": ok, "results": results, "timeout": tmo, "ipc_ops": c.ipc_ops,
                          "ops": dict(c.ops), "inner_tensor_ops": c.inner_tensor_ops,
                          "ms_per_10MB_allreduce": round(el * 1e3, 4)}), flush=True)
    else:
        print(json.dumps({"rank": r, "results": results}), file=sys.stderr, flush=True)
    ctx.shutdown()
    return 0 if ok and not tmo else 1


if __name__ == "__main__":
    sys.exit(main())
