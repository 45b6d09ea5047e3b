"""Summarise a rocprofv3 --stats kernel_stats.csv: per-kernel total/avg time and per-step share.

    python tools/prof_summary.py gpurun_out/prof1/run_kernel_stats.csv [--steps 25]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=0, help="timed+warmup steps in the profiled run")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'total_ms':>9} {'pct':>6} {'calls':>6} {'avg_us':>8} {'per_step_us':>11}  kernel")
    for r in rows:
        t = float(r["TotalDurationNs"])
        ps = t / a.steps / 1e3 if a.steps else 0.0
        name = r["Name"].replace("(anonymous namespace)::", "")
        name = name.split("(")[0] if not name.startswith("void") else name[5:].split("(")[0]
        print(f"{t / 1e6:9.3f} {float(r['Percentage']):6.2f} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:8.1f} "
              f"{ps:11.1f}  {name[:90]}")
    print(f"sum of kernel time: {tot / 1e6:.3f} ms" + (f"  ({tot / a.steps / 1e6:.3f} ms/step)" if a.steps else ""))


if __name__ == "__main__":
    main()
