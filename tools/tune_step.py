"""Tune the conv configurations of the VGG training step IN the step, not in isolation.

tools/tune_convs.py times every (tile, split-K, row order) of a conv call alone.  In the step the
backward runs on two streams (data gradients + BN backward on one, weight gradients + their split-K
reductions on the other) that share the CUs, HBM and L2, so the fastest isolated configuration is
not always the fastest in context (e.g. a wgrad with many splits runs its conv quickly but streams
hundreds of MB of split-K slabs through the memory system the critical path needs).

For every conv call of the step (one table key may cover several layers of the same shape) this
keeps the ``--top`` best isolated candidates and picks, by coordinate descent, the one that gives
the lowest whole-step time (median of ``--reps`` runs of ``--steps`` steps).  A candidate must win
by ``--min-gain`` (relative) to replace the current choice.  The result is merged into
distributed_pytorch_amd/tuning/mi355x.json ([tile, splits, posmajor, isolated_ms]).

    python tools/tune_step.py [--batch 256] [--impl x3] [--top 5] [--kinds wgrad,dgrad,fprop] [--per-split]

``--per-split``: the candidates of a call are the fastest isolated configuration of EVERY split-K
count instead of the ``--top`` fastest overall.  The isolated ranking favours many splits (short
conv, long slab reduction); on the weight-gradient stream, which shares the chip with the critical
path, a configuration with fewer splits can win in the step although it loses alone.

Precision gate (default on; ``--no-precision`` skips it): a plan changes the
order and split of a conv's reduction, and with fp16-pair (h2) operands that moves the step's
gradient errors (round 5: two faster candidate sets failed the parity suite afterwards).  So every
candidate that wins on time is also scored BEFORE it is accepted: one batch-256 training step with
the candidate plan installed, from the random init and from a trained state (200 training steps),
each against fp64 autograd of the same step (tests/test_parity256_gpu.py's fixture).  It is
accepted only if, at both states, the median tensor's error (relative to torch fp32's) grows by at
most ``--gate-slack`` (default 10 %) over the starting table's, and at the random init it stays
within ``--gate-median`` (1.3; the suite's bound is 1.5) with every tensor within 4x of the floor.
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from distributed_pytorch_amd.engine import conv_key  # noqa: E402
from distributed_pytorch_amd.parallel import NullComm  # noqa: E402


def step_ms(step, steps, reps):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) / steps * 1e3)
    return statistics.median(out)


def isolated(e, i, kind, n, iters=3):
    """[(ms, (tile, eff_splits, pm))] for every candidate of conv call (i, kind), fastest first."""
    l = e.spec.convs[i]
    impl = e._layer_impl(i)
    key = (impl, kind, n, i)
    saved = e._cfg_cache.get(key)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for tile, s, pm in e.conv_candidates(i, kind):
        M = n * l.hw * l.hw
        red = M if kind == "wgrad" else 9 * (l.cin_pad if kind == "fprop" else l.cout)
        s = e.K.conv_splits(red, s) if impl == "fp32" else e.K.x3_splits(red, s)
        cand = (tile, s, pm)
        if any(c == cand for _, c in res):
            continue
        e._cfg_cache[key] = cand
        if e._slab_need(i, kind, n) * 4 > (256 << 20):
            continue
        fn = {"fprop": lambda: e._conv_fwd(i, e.x0[:n], n, reduce=False),
              "dgrad": lambda: e._conv_dgrad(i, n),
              "wgrad": lambda: e._conv_wgrad(i, e.x0[:n], n)}[kind]
        fn()
        ev0.record()
        for _ in range(iters):
            fn()
        ev1.record()
        torch.cuda.synchronize()
        res.append((ev0.elapsed_time(ev1) / iters, cand))
    if saved is not None:
        e._cfg_cache[key] = saved
    return sorted(res)


class PrecisionGate:
    """Scores a plan table (the tuning engine's ``_cfg_cache``) against fp64 autograd at batch 256,
    from the random init and from a trained state, with the parity suite's own fixture."""

    def __init__(self, impl, gate_median=1.3, trained_steps=200, slack=0.10):
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import test_parity256_gpu as P  # noqa: E402  (the suite's fixture, not a copy of it)

        self.P, self.impl, self.gate_median, self.slack = P, impl, gate_median, slack
        self.base = None  # per-reference medians of the starting table (set by the first score)
        self.refs = [P._reference()]
        if trained_steps:
            self.refs.append(P._reference(P._trained_state(trained_steps), data_seed=512))
        self.floor, self.tref = [], []
        for ref in self.refs:
            tg, _ = P._torch_fp32_errors(ref)
            pert = ([P._perturbed_errors(ref, sd, torch.float64) for sd in (1, 2)]
                    + [P._perturbed_errors(ref, sd, torch.float32) for sd in (3, 4)])
            self.tref.append(tg)
            self.floor.append({n: (None if e is None else max([e] + [p[n] for p in pert])) for n, e in tg.items()})

    def score(self, cfg_cache):
        """{"median": worst median ratio vs torch fp32, "worst_floor": worst ratio to the floor, "ok": bool}"""
        from distributed_pytorch_amd.engine import VGGEngine

        med, worst, per, worst0 = 0.0, 0.0, [], 0.0
        for ri, (ref, floor, tref) in enumerate(zip(self.refs, self.floor, self.tref)):
            e = VGGEngine("VGG11", "cuda", max_batch=self.P.N, impl=self.impl)
            e._cfg_cache.update({k: v for k, v in cfg_cache.items() if k[2] == self.P.N})
            e.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in ref["sd0"].items()})
            x4 = torch.zeros(self.P.N, 32, 32, 4)
            x4[..., :3] = ref["x"].float().permute(0, 2, 3, 1)
            e.forward_backward(x4.cuda(), ref["t"].cuda())
            torch.cuda.synchronize()
            e.check_signals()
            ratios = []
            for n, gref in ref["grads"].items():
                if gref.abs().max() < 1e-7:
                    continue
                err = self.P._rel(e._to_torch_layout(n, e.grads[n]).cpu(), gref)
                worst = max(worst, err / (floor[n] + 1e-5 / 4.0))
                if ri == 0:
                    worst0 = max(worst0, err / (floor[n] + 1e-5 / 4.0))
                ratios.append(err / max(tref[n], 1e-12))
            ratios.sort()
            med = max(med, ratios[len(ratios) // 2])
            per.append(round(ratios[len(ratios) // 2], 3))
            del e
        if self.base is None:
            self.base = per
        ok = (all(m <= b * (1.0 + self.slack) for m, b in zip(per, self.base))
              and per[0] <= self.gate_median and worst0 <= 4.0)
        return {"median": round(med, 3), "worst_floor": round(worst, 3), "per_ref_median": per, "ok": ok}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--impl", default="x3")
    ap.add_argument("--top", type=int, default=5)
    ap.add_argument("--steps", type=int, default=15)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--min-gain", type=float, default=0.004)
    ap.add_argument("--kinds", default="wgrad,dgrad,fprop")
    ap.add_argument("--out", default=os.path.join(ROOT, "distributed_pytorch_amd", "tuning", "mi355x.json"))
    ap.add_argument("--dry-run", action="store_true", help="report, do not write the table")
    ap.add_argument("--per-split", action="store_true",
                    help="candidates: the fastest isolated config of every split count (not the --top overall)")
    ap.add_argument("--no-precision", action="store_true", help="skip the precision gate (timing only)")
    ap.add_argument("--gate-median", type=float, default=1.3)
    ap.add_argument("--gate-slack", type=float, default=0.10)
    a = ap.parse_args()
    args = bench.parse(["--batch", str(a.batch), "--impl", a.impl])
    dev = torch.device("cuda", 0)
    engine, sync, it = bench.build(args, dev, 0, 1, NullComm())
    step = bench.make_step(engine, sync, it)
    for _ in range(10):
        step()
    n = a.batch
    base = step_ms(step, a.steps, a.reps)
    print(json.dumps({"start_step_ms": round(base, 4)}), flush=True)
    gate = None if a.no_precision else PrecisionGate(a.impl, a.gate_median, slack=a.gate_slack)
    if gate is not None:
        g0 = gate.score(engine._cfg_cache)
        print(json.dumps({"start_precision": g0}), flush=True)
    rejected = {}
    # group layers by table key (layers of identical shape share one entry)
    groups = {}
    for kind in a.kinds.split(","):
        for i, l in enumerate(engine.spec.convs):
            if kind == "dgrad" and i == 0:
                continue
            k = conv_key(engine._layer_impl(i), kind, n, l.hw, l.cin_pad, l.cout)
            groups.setdefault(k, (kind, []))[1].append(i)
    table = json.load(open(a.out)) if os.path.exists(a.out) else {}
    changed = {}
    for k, (kind, layers) in groups.items():
        i0 = layers[0]
        cands = isolated(engine, i0, kind, n)
        cur = engine.conv_config(i0, kind, n)
        if a.per_split:
            seen, top = set(), []
            for _, c in cands:  # fastest first: keep the best config of each split count
                if c[1] not in seen:
                    seen.add(c[1])
                    if c != cur:
                        top.append(c)
        else:
            top = [c for _, c in cands[: a.top] if c != cur]
        iso = {c: ms for ms, c in cands}
        cur_ms = step_ms(step, a.steps, a.reps)
        best, best_ms = cur, cur_ms
        for c in top:
            for i in layers:
                engine._cfg_cache[(engine._layer_impl(i), kind, n, i)] = c
            for _ in range(2):
                step()
            ms = step_ms(step, a.steps, a.reps)
            print(f"  {k} {c} iso={iso.get(c, 0):.4f} step={ms:.4f} (cur {cur} {cur_ms:.4f})", flush=True)
            if ms < best_ms * (1 - a.min_gain):
                if gate is not None:  # faster: is it still fp32-grade?
                    sc = gate.score(engine._cfg_cache)
                    print(f"    precision {sc}", flush=True)
                    if not sc["ok"]:
                        rejected.setdefault(k, []).append([list(c), round(ms, 4), sc])
                        continue
                best, best_ms = c, ms
        for i in layers:
            engine._cfg_cache[(engine._layer_impl(i), kind, n, i)] = best
        for _ in range(2):
            step()
        if best != cur:
            changed[k] = [best[0], best[1], int(best[2]), iso.get(best, 0.0)]
        print(json.dumps({"key": k, "layers": layers, "choice": list(best), "was": list(cur),
                          "step_ms": round(best_ms, 4), "was_ms": round(cur_ms, 4)}), flush=True)
    final = step_ms(step, a.steps, a.reps * 2)
    out = {"start_step_ms": round(base, 4), "final_step_ms": round(final, 4), "changed": changed,
           "rejected_on_precision": rejected}
    if gate is not None:
        out["final_precision"] = gate.score(engine._cfg_cache)
    print(json.dumps(out), flush=True)
    if changed and not a.dry_run:
        table.update(changed)
        with open(a.out, "w") as f:
            json.dump(table, f, indent=0, sort_keys=True)
        print("wrote", a.out, flush=True)


if __name__ == "__main__":
    main()
