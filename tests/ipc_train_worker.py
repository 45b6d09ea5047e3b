"""One rank of the multi-rank training determinism probe (ranks share one GPU, peer-memory
collectives): VGG-11 steps with per-step float64 checksums of the local gradients (before the
all-reduce), the reduced gradients and the parameters, printed by rank 0 as one JSON line.

DPA_TRAIN_PROBE_MODE=serial: forward_backward with no hooks, host sync, all-reduce, host sync,
update (nothing overlaps); =overlap: the DDP strategy as the bench runs it (bucket collectives
during backward), checksums after each step only.  Two runs of the same mode must print the same
numbers: a difference localises a race (compute vs communication)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_amd.data import DeviceLoader, ShardSampler, synthetic_cifar  # noqa: E402
from distributed_pytorch_amd.engine import VGGEngine  # noqa: E402
from distributed_pytorch_amd.parallel import init_env, make_sync  # noqa: E402


def cs(t):
    return float(t.double().sum().item())


def main():
    os.environ.setdefault("DPA_IPC_BLOCKS", "16")
    ctx = init_env(comm="ipc")
    dev, W, r, c = ctx.device, ctx.world, ctx.rank, ctx.comm
    mode = os.environ.get("DPA_TRAIN_PROBE_MODE", "serial")
    impl = os.environ.get("DPA_TRAIN_PROBE_IMPL", "x3")
    steps = int(os.environ.get("DPA_TRAIN_PROBE_STEPS", "6"))
    batch = 64
    ds = synthetic_cifar(4096, 0)
    ld = DeviceLoader(ds, batch, dev, sampler=ShardSampler(len(ds), W, r, shuffle=True, seed=0), train=True,
                      seed=7919 + r, drop_last=True)
    e = VGGEngine("VGG11", dev, max_batch=batch, impl=impl)
    e.init_parameters(seed=1)
    sync = make_sync("ddp", e, c, bucket_mb=10.0, overlap=(mode == "overlap"))
    it = iter(ld)
    rows = []
    for s in range(steps):
        x, t = next(it)
        if mode == "serial":
            e.forward_backward(x, t)
            torch.cuda.synchronize(dev)
            loc = cs(e.grads.flat)
            with c.region():
                c.all_reduce(e.grads.flat)
            c.wait()
            torch.cuda.synchronize(dev)
            red = cs(e.grads.flat)
            e.sgd_step(1.0 / W)
        else:
            sync.begin_step()
            e.forward_backward(x, t, grad_ready=sync.grad_ready, pre_forward=sync.pre_forward,
                               params_free=sync.params_free)
            sync.update(sync.finish())
            loc = None
            red = None
        e.finish_step()
        torch.cuda.synchronize(dev)
        rows.append({"step": s, "loss": float(e.loss.item()), "local": loc, "reduced": red,
                     "params": cs(e.params.flat)})
    e.check_signals()
    tmo = c.timed_out()
    if r == 0:
        print(json.dumps({"mode": mode, "impl": impl, "world": W, "timeout": tmo, "rows": rows}), flush=True)
    else:
        print(json.dumps({"rank": r, "local": [x["local"] for x in rows]}), flush=True)
    ctx.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
