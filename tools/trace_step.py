"""Print one training step's kernel timeline from a rocprofv3 --kernel-trace CSV or rocpd database.

    python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv [--step -3] [--filter bn_]
    python tools/trace_step.py gpurun_out/prof/run_results.db
Steps are delimited by the SGD kernel.
"""
import argparse
import csv
import sqlite3


def load_rows(path):
    """Kernel records as dicts with the CSV trace's column names, start-time order."""
    if not path.endswith(".db"):
        return sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    con = sqlite3.connect(path)
    q = "select name, start, end, grid_x, grid_y, stream_id from kernels order by start"
    rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e, "Grid_Size_X": gx, "Grid_Size_Y": gy,
             "Stream_Id": sid} for n, s, e, gx, gy, sid in con.execute(q)]
    con.close()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--step", type=int, default=-3)
    ap.add_argument("--filter", default="")
    ap.add_argument("--marker", default="sgd_flat")
    a = ap.parse_args()
    rows = load_rows(a.csv)
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    i0, i1 = idx[a.step - 1], idx[a.step]
    t0 = int(rows[i0 + 1]["Start_Timestamp"])
    prev_end = t0
    for r in rows[i0 + 1:i1 + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if a.filter in name:
            print(f"{(s - t0) / 1e3:9.1f} gap{(s - prev_end) / 1e3:6.1f} dur{(e - s) / 1e3:8.1f}  grid={r['Grid_Size_X']:>8}x{r['Grid_Size_Y']:<4} s{r.get('Stream_Id', '')!s:<2} {name[:70]}")
        prev_end = e
    print(f"step span {(int(rows[i1]['End_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
