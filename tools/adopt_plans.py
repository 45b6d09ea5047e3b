"""Gated adoption of candidate conv plans into the tuning table (tools/tune_step.py's precision gate,
without its isolated search): candidates come from a JSON file ({conv_key: [tile, splits, pm, ms]},
e.g. tools/halo64_ab.py's best plans).  In the order of the file, each candidate is installed into
the running VGG step, scored against fp64 autograd at the random init and at a trained state
(PrecisionGate: median tensor error relative to torch fp32 may grow by at most ``--gate-slack`` over
the STARTING table's, the random-init median stays <= ``--gate-median``, every tensor within 4x of
the floor) and kept only if it passes AND the step gets faster by ``--min-gain``.  The final table is
timed against the starting one in interleaved rounds.

    python tools/adopt_plans.py --cands distributed_pytorch_amd/tuning/halo64_extra.json --impl h2 [--write]
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
from distributed_pytorch_amd.engine import conv_key  # noqa: E402
from distributed_pytorch_amd.parallel import NullComm  # noqa: E402
from tune_step import PrecisionGate, step_ms  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cands", required=True)
    ap.add_argument("--impl", default="h2")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--min-gain", type=float, default=0.002)
    ap.add_argument("--gate-median", type=float, default=1.3)
    ap.add_argument("--gate-slack", type=float, default=0.10)
    ap.add_argument("--out", default=os.path.join(ROOT, "distributed_pytorch_amd", "tuning", "mi355x.json"))
    ap.add_argument("--write", action="store_true", help="merge the accepted plans into --out")
    ap.add_argument("--log", default=os.path.join(ROOT, "gpurun_out", "adopt_plans.json"))
    a = ap.parse_args()
    cands = json.load(open(a.cands))
    args = bench.parse(["--batch", str(a.batch), "--impl", a.impl])
    engine, sync, it = bench.build(args, torch.device("cuda", 0), 0, 1, NullComm())
    step = bench.make_step(engine, sync, it)
    for _ in range(10):
        step()
    n = a.batch
    keys = {}  # conv_key -> [(cache key)] of the layers it covers
    for i, l in enumerate(engine.spec.convs):
        for kind in ("fprop", "dgrad", "wgrad"):
            if kind == "dgrad" and i == 0:
                continue
            impl = engine._layer_impl(i)
            keys.setdefault(conv_key(impl, kind, n, l.hw, l.cin_pad, l.cout), []).append((impl, kind, n, i))
            engine.conv_config(i, kind, n)  # populate the cache with the current plan
    start = {k: engine._cfg_cache[ck[0]] for k, ck in keys.items()}
    gate = PrecisionGate(a.impl, a.gate_median, slack=a.gate_slack)
    g0 = gate.score(engine._cfg_cache)
    cur_ms = step_ms(step, a.steps, a.reps)
    log = {"start_precision": g0, "start_step_ms": round(cur_ms, 4), "steps": []}
    print(json.dumps(log), flush=True)
    accepted = {}
    for k, vs in cands.items():
        if k not in keys:
            continue
        if not isinstance(vs[0], list):  # one plan, or a list of alternatives (first kept wins)
            vs = [vs]
        old = engine._cfg_cache[keys[k][0]]
        for v in vs:
            c = (int(v[0]), int(v[1]), int(v[2]))
            if c == old:
                continue
            for ck in keys[k]:
                engine._cfg_cache[ck] = c
            sc = gate.score(engine._cfg_cache)
            for _ in range(3):
                step()
            ms = step_ms(step, a.steps, a.reps) if sc["ok"] else None
            keep = sc["ok"] and ms < cur_ms * (1 - a.min_gain)
            rec = {"key": k, "cand": list(c), "was": list(old), "precision": sc, "step_ms": ms and round(ms, 4),
                   "was_ms": round(cur_ms, 4), "kept": keep}
            log["steps"].append(rec)
            print(json.dumps(rec), flush=True)
            if keep:
                accepted[k] = [c[0], c[1], c[2], float(v[3]) if len(v) > 3 else 0.0]
                cur_ms = ms
                break
            for ck in keys[k]:
                engine._cfg_cache[ck] = old
    final = dict(engine._cfg_cache)
    # interleaved start / final timing
    t_start, t_final = [], []
    for _ in range(4):
        for tab, acc in ((start, t_start), (None, t_final)):
            for k, ck in keys.items():
                for c in ck:
                    engine._cfg_cache[c] = tab[k] if tab is not None else final[c]
            for _ in range(3):
                step()
            acc.append(step_ms(step, a.steps, a.reps))
    log.update(accepted=accepted, final_precision=gate.score(final),
               start_ms=[round(x, 4) for x in t_start], final_ms=[round(x, 4) for x in t_final],
               gain=round(statistics.median(t_start) / statistics.median(t_final) - 1, 4))
    print(json.dumps({k: log[k] for k in ("accepted", "final_precision", "start_ms", "final_ms", "gain")}), flush=True)
    os.makedirs(os.path.dirname(a.log), exist_ok=True)
    with open(a.log, "w") as f:
        json.dump(log, f, indent=1)
    if a.write and accepted:
        table = json.load(open(a.out)) if os.path.exists(a.out) else {}
        table.update(accepted)
        with open(a.out, "w") as f:
            json.dump(table, f, indent=0, sort_keys=True)
        print("wrote", a.out, flush=True)


if __name__ == "__main__":
    main()
