"""Differential re-execution: is one process's training step deterministic while OTHER processes
load the same GPU?  (VERDICT r5 "what's missing" #1: several processes sharing one GPU are not
run-to-run reproducible.)

Every child runs the bench's own 1-rank training step (bench.make_step: augment once, forward,
backward on two streams with kernel-start signals, fused SGD) from a snapshot of the training
state, hashes every buffer the step wrote (per layer, in execution order), restores the snapshot
and runs the identical step again.  The engine is deterministic, so the two hash vectors must be
equal; the first buffer (in execution order) that differs names the producer that read stale or
partly written data.  No communication between the processes: the others only supply the load.

    python tools/replay_check.py --procs 4 --pairs 150 --batch 64 [--impl h2] [--env K=V,...]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _bufs(engine):
    """(name, tensor) of every buffer a training step writes, in execution order."""
    out = []
    L = engine.spec.convs
    for i in range(len(L)):
        out.append((f"z{i}", engine.z[i]))
        if engine.a3[i] is not None:
            out.append((f"a3_{i}", engine.a3[i]))
        if engine.a[i] is not None:
            out.append((f"a{i}", engine.a[i]))
        out.append((f"stats{i}", torch.cat([engine.stats[i][k] for k in ("mean", "invstd", "scale", "shift")])))
    out.append(("loss", engine.loss))
    out.append(("dlogits", engine.dlogits))
    for i in range(len(L) - 1, -1, -1):
        out.append((f"g{i}", engine.g[i]))
        if engine.dz3[i] is not None:
            out.append((f"dz3_{i}", engine.dz3[i]))
        if engine.dz[i] is not None:
            out.append((f"dz{i}", engine.dz[i]))
        l = L[i]
        for nm in (f"{l.conv_key}.weight", f"{l.conv_key}.bias", f"{l.bn_key}.weight", f"{l.bn_key}.bias"):
            out.append((f"grad:{nm}", engine.grads[nm]))
    out.append(("grad:fc1", torch.cat([engine.grads["fc1.weight"].flatten(), engine.grads["fc1.bias"]])))
    out.append(("params", engine.params.flat))
    out.append(("mom", engine.mom.flat))
    out.append(("buffers", engine.buffers.flat))
    if engine.wplanes is not None:
        out.append(("wplanes", engine.wplanes))
    return out


def _hash(t):
    v = t.contiguous().view(-1)
    if v.element_size() == 2:
        v = v.view(torch.int16).to(torch.int32)
    elif v.element_size() == 8:
        v = v.view(torch.int32)
    else:
        v = v.view(torch.int32)
    # position-weighted, so a permutation or a swapped pair also shows
    w = (torch.arange(v.numel(), device=v.device, dtype=torch.int64) % 1021) + 1
    return (v.to(torch.int64) * w).sum()


def _conv0_ref(x, w):
    import torch.nn.functional as F

    xd = x[..., :3].double().permute(0, 3, 1, 2)
    wd = w[..., :3].double().permute(0, 3, 1, 2)
    return F.conv2d(xd, wd, padding=1).permute(0, 2, 3, 1)


def _diag_conv0(x, w_snap, z, cands) -> dict:
    """Where a first-layer output z (computed from x and the pre-step weights w_snap) is wrong, and
    whether the wrong values are those of an OLDER weight tensor (cands: name -> weights), i.e. a
    stale read of w.  conv0_fwd_kernel's block = (image, 8-row band), thread = (channel quad, pixel
    lane)."""
    ref = _conv0_ref(x, w_snap)
    tol = 1e-4 * float(ref.abs().max())
    bad = (z.double() - ref).abs() > tol
    idx = bad.nonzero().cpu()
    out = {"wrong": int(idx.shape[0])}
    if not idx.shape[0]:
        return out
    zb = z.double()[bad]
    for nm, w in cands.items():  # wrong values explained by another weight tensor
        r2 = _conv0_ref(x, w)[bad]
        out[f"match_{nm}"] = int(((zb - r2).abs() <= tol).sum())
    blk = idx[:, 0] * 4 + idx[:, 1] // 8
    out["blocks"] = sorted(set(blk.tolist()))[:24]
    out["n_blocks"] = len(set(blk.tolist()))
    out["channels"] = sorted(set(idx[:, 3].tolist()))[:64]
    out["pixels"] = len(set((idx[:, 0] * 1024 + idx[:, 1] * 32 + idx[:, 2]).tolist()))
    per = {}
    for b, c, h, w_ in zip(blk.tolist(), idx[:, 3].tolist(), idx[:, 1].tolist(), idx[:, 2].tolist()):
        e = per.setdefault(b, [set(), set()])
        e[0].add(c)
        e[1].add((h % 8) * 32 + w_)
    out["per_block"] = {str(b): {"ch": sorted(v[0])[:16], "nch": len(v[0]), "npix": len(v[1]),
                                 "pix": sorted(v[1])[:12]} for b, v in list(per.items())[:6]}
    return out


def child(a) -> dict:
    import bench
    from distributed_pytorch_amd.data import DeviceLoader, ShardSampler, synthetic_cifar
    from distributed_pytorch_amd.engine import VGGEngine
    from distributed_pytorch_amd.parallel import NullComm, make_sync

    dev = torch.device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    train = synthetic_cifar(4096, 0)
    loader = DeviceLoader(train, a.batch, dev, sampler=ShardSampler(len(train), 1, 0, shuffle=True, seed=0),
                          train=True, seed=7919, drop_last=True)
    engine = VGGEngine("VGG11", dev, max_batch=a.batch, impl=a.impl)
    engine.init_parameters(seed=1)
    sync = make_sync("ddp", engine, NullComm())
    batches = iter(loader)
    x, t = next(batches)
    x, t = x.clone(), t.clone()

    def fixed():
        while True:
            yield x, t

    step = bench.make_step(engine, sync, fixed())
    for _ in range(3):  # warm: past the first-step (no momentum) path
        step()
    names = [n for n, _ in _bufs(engine)]
    state = (engine.params.flat, engine.mom.flat, engine.buffers.flat, engine.nbt, engine.loss_accum)
    hashes, pre, zdiff = [], [], []
    diag_out = []
    w0 = engine.params["layers.0.weight"]
    z0 = engine.z[0]
    nblk = z0.shape[0] * 4  # conv0 blocks: (image, 8-row band)
    blk_hits = torch.zeros(nblk, dtype=torch.int64, device=dev)
    t0 = time.time()
    pairs = 0
    w_prev = w0.clone()
    while pairs < a.pairs and time.time() - t0 < a.seconds:
        snap = [s.clone() for s in state]
        w_snap = w0.clone() if a.diag else None
        taken = engine.steps_taken
        pair, pp = [], []
        for rep in range(2):
            if rep:
                for d, s in zip(state, snap):
                    d.copy_(s)
                engine.steps_taken = taken
                engine.refresh_weight_planes()
            pp.append(torch.stack([_hash(x), _hash(w0)]))  # conv0's inputs, right before the step
            step()
            if rep == 0:
                z0a = z0.clone()
                w_after0 = w0.clone() if a.diag else None
            else:
                d = (z0 != z0a)
                if a.diag and len(diag_out) < 4 and bool(d.any()):  # (synchronises: diagnostic runs only)
                    diag_out.append({"pair": pairs,
                                     "rep0": _diag_conv0(x, w_snap, z0a, {"prev_snap": w_prev}),
                                     "rep1": _diag_conv0(x, w_snap, z0, {"after_rep0": w_after0})})
                blk_hits += d.view(nblk, -1).any(dim=1).long()
                zdiff.append(torch.stack([d.sum().double(), (z0 - z0a).abs().max().double(),
                                          z0a.abs().max().double()]))
            pair.append(torch.stack([_hash(b) for _, b in _bufs(engine)]))
        hashes.append(torch.stack(pair))
        pre.append(torch.stack(pp))
        if a.diag:
            w_prev = w_snap
        pairs += 1
        if pairs % 25 == 0 and dev.type == "cuda":
            torch.cuda.synchronize()
    if dev.type == "cuda":
        torch.cuda.synchronize()
        engine.check_signals()
    H = torch.stack(hashes).cpu()  # [pairs, 2, nbuf]
    P = torch.stack(pre).cpu()  # [pairs, 2 reps, (x, w0)]
    Z = torch.stack(zdiff).cpu()  # [pairs, (elements differing, max |diff|, max |z0|)]
    diff = (H[:, 0] != H[:, 1])
    bad_pairs = diff.any(dim=1).nonzero().flatten().tolist()
    first = {}
    for p in bad_pairs:
        idx = diff[p].nonzero().flatten().tolist()
        first[p] = [names[j] for j in idx[:3]]
    hits = blk_hits.cpu()
    by_xcd = [int(hits[x::8].sum()) for x in range(8)]  # round-robin dispatch: block b on XCD b % 8
    return {"rank": a.rank, "pairs": pairs, "bad_pairs": len(bad_pairs),
            "inputs_differ": int((P[:, 0] != P[:, 1]).any(dim=1).sum()),
            "z0_bad_pairs": int((Z[:, 0] > 0).sum()),
            "z0_elems_differing": [int(v) for v in Z[Z[:, 0] > 0][:6, 0].tolist()],
            "z0_maxdiff_vs_max": [[float(f"{u:.3g}"), float(f"{v:.3g}")] for u, v in Z[Z[:, 0] > 0][:4, 1:].tolist()],
            "z0_block_hits_by_xcd": by_xcd, "z0_blocks_hit": int((hits > 0).sum()), "z0_blocks": nblk,
            "first_diffs": {str(k): v for k, v in list(first.items())[:4]}, "diag": diag_out}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--pairs", type=int, default=150)
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--impl", default="h2")
    ap.add_argument("--env", default="", help="comma list K=V for the children (A/B of engine switches)")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--diag", action="store_true", help="locate the wrong first-layer outputs of bad pairs")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--rank", type=int, default=0)
    a = ap.parse_args(argv)
    if a.child:
        print(json.dumps(child(a)), flush=True)
        return 0
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for kv in filter(None, a.env.split(",")):
        k, v = kv.split("=", 1)
        env[k] = v
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", "--rank", str(r), "--pairs",
                               str(a.pairs), "--seconds", str(a.seconds), "--batch", str(a.batch), "--impl", a.impl, "--device", a.device]
                              + (["--diag"] if a.diag else []),
                              stdout=subprocess.PIPE, env=env, text=True) for r in range(a.procs)]
    rows, rc = [], 0
    for p in procs:
        out, _ = p.communicate(timeout=a.seconds + 300)
        rc = rc or p.returncode
        rows += [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    print(json.dumps({"procs": a.procs, "impl": a.impl, "env": a.env, "rows": rows,
                      "bad_pairs_total": sum(r["bad_pairs"] for r in rows)}), flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
