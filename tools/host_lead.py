"""Host lead per kernel from a rocprofv3 ``--kernel-trace --hip-runtime-trace`` database: for each
kernel of one step, when its launch call returned on the host and when it started on the GPU.
A kernel that starts right after its launch call returned (lead ~0) was waiting for the host.

    python tools/host_lead.py gpurun_out/prof/run_results.db [--marker augment] [--step -2] [--api-min-us 20]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="augment")
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--api-min-us", type=float, default=20.0, help="also list host API calls longer than this")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    ks = con.execute("select name, start, end, stream_id, stack_id from kernels order by start").fetchall()
    api = {r[0]: r[1:] for r in con.execute("select stack_id, name, start, end from regions")}
    idx = [i for i, k in enumerate(ks) if a.marker in k[0]]
    i0, i1 = idx[a.step - 1], idx[a.step]
    t0 = ks[i0][1]
    print(f"{'gpu_start':>9} {'dur':>6} {'host_ret':>9} {'lead':>7} st  kernel")
    for name, s, e, sid, corr in ks[i0:i1]:
        h = api.get(corr)
        hr = (h[2] - t0) / 1e3 if h else float("nan")
        n = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:6.1f} {hr:9.1f} {(s - h[2]) / 1e3 if h else float('nan'):7.1f} s{sid:<2} {n}")
    t1 = ks[i1][1]
    print("long host API calls in the step:")
    for name, s, e in con.execute("select name, start, end from regions where start >= ? and start < ? "
                                  "and (end - start) > ? order by start", (t0, t1, int(a.api_min_us * 1e3))):
        print(f"  {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} us  {name}")


if __name__ == "__main__":
    main()
