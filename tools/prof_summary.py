"""Summarise a rocprofv3 kernel trace: per-kernel total/avg time and per-step share.

Accepts the ``--stats --output-format csv`` file (``*_kernel_stats.csv``) or the default rocpd
SQLite database (``*_results.db``, read through its ``kernels`` view).

    python tools/prof_summary.py gpurun_out/prof1/run_kernel_stats.csv [--steps 25]
    python tools/prof_summary.py gpurun_out/val_prof/val_results.db --steps 35
"""
import argparse
import csv
import sqlite3
from collections import defaultdict


def _short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0] if not name.startswith("void") else name[5:].split("(")[0]


def rows_from_db(path):
    """[(name, calls, total_ns)] from a rocpd database, largest total first."""
    acc = defaultdict(lambda: [0, 0])
    con = sqlite3.connect(path)
    for name, dur in con.execute("select name, duration from kernels"):
        a = acc[name]
        a[0] += 1
        a[1] += int(dur)
    con.close()
    return sorted(((n, c, t) for n, (c, t) in acc.items()), key=lambda r: -r[2])


def rows_from_csv(path):
    return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(path))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=0, help="timed+warmup steps in the profiled run")
    ap.add_argument("--top", type=int, default=0, help="print only the N largest kernels")
    a = ap.parse_args()
    rows = rows_from_db(a.path) if a.path.endswith(".db") else rows_from_csv(a.path)
    tot = sum(t for _, _, t in rows)
    print(f"{'total_ms':>9} {'pct':>6} {'calls':>6} {'avg_us':>8} {'per_step_us':>11}  kernel")
    for name, calls, t in rows[: a.top or None]:
        ps = t / a.steps / 1e3 if a.steps else 0.0
        print(f"{t / 1e6:9.3f} {100.0 * t / tot:6.2f} {calls:>6} {t / calls / 1e3:8.1f} {ps:11.1f}  {_short(name)[:90]}")
    print(f"sum of kernel time: {tot / 1e6:.3f} ms" + (f"  ({tot / a.steps / 1e6:.3f} ms/step)" if a.steps else ""))


if __name__ == "__main__":
    main()
