"""Per-tensor gradient error table of one batch-256 training step vs fp64 autograd, for every conv
arithmetic (fp32 / x3 / h2), from the random init and from the trained state of
tests/test_parity256_gpu.py (its own fixture): error / torch-fp32 error per tensor, the medians the
suite bounds, and the step's error floor.

    python tools/parity_report.py [--impls fp32,x3,h2] [--out gpurun_out/parity_report.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impls", default="fp32,x3,h2")
    ap.add_argument("--out", default="gpurun_out/parity_report.json")
    a = ap.parse_args()
    import test_parity256_gpu as P

    impls = tuple(a.impls.split(","))
    rep = {}
    for name, ref in (("init", P._reference()), ("trained", P._reference(P._trained_state(), data_seed=512))):
        e = P._errors(ref, impls=impls, dump=f"gpurun_out/parity_{name}.json")
        tref, floor = e["torch_fp32"]["grads"], e["floor"]
        rows = {n: {"torch_fp32": t, "floor": floor[n], **{i: e[i]["grads"][n] for i in impls}}
                for n, t in tref.items() if t is not None}
        med = {}
        for i in impls:
            r = sorted(rows[n][i] / max(rows[n]["torch_fp32"], 1e-12) for n in rows)
            med[i] = {"median_ratio": round(r[len(r) // 2], 3), "max_ratio": round(r[-1], 2),
                      "worst_vs_floor": round(max(rows[n][i] / (rows[n]["floor"] + 2.5e-6) for n in rows), 2),
                      "loss_rel": e[i]["loss"]}
        rep[name] = {"summary": med, "tensors": rows}
        print(name, json.dumps(med), flush=True)
        print(f"{'tensor':20s} {'torch32':>9s} " + " ".join(f"{i:>9s}" for i in impls) + "  (ratios to torch fp32)")
        for n, r in rows.items():
            print(f"{n:20s} {r['torch_fp32']:9.2e} " + " ".join(f"{r[i] / max(r['torch_fp32'], 1e-12):9.2f}" for i in impls))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
