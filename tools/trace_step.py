"""Print one training step's kernel timeline from a rocprofv3 --kernel-trace CSV.

    python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv [--step -3] [--filter bn_]
Steps are delimited by the SGD kernel.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--step", type=int, default=-3)
    ap.add_argument("--filter", default="")
    ap.add_argument("--marker", default="sgd_flat")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    i0, i1 = idx[a.step - 1], idx[a.step]
    t0 = int(rows[i0 + 1]["Start_Timestamp"])
    prev_end = t0
    for r in rows[i0 + 1:i1 + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if a.filter in name:
            print(f"{(s - t0) / 1e3:9.1f} gap{(s - prev_end) / 1e3:6.1f} dur{(e - s) / 1e3:8.1f}  grid={r['Grid_Size_X']:>8}x{r['Grid_Size_Y']:<4} {name[:70]}")
        prev_end = e
    print(f"step span {(int(rows[i1]['End_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
