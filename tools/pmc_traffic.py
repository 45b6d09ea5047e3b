"""Per-kernel HBM traffic of one step from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
(scripts/gpu_resnet_pmc.sh): kernel-time sum, GB read / written (the counters are in KB), and the
achieved rate; plus MFMA-busy cycles from the SQ pass.

    python tools/pmc_traffic.py gpurun_out/rnp_A gpurun_out/rnp_C gpurun_out/rnp_D [--top 30]
"""
import argparse
import collections
import csv
import re


def load(path):
    d = collections.OrderedDict()
    for r in csv.DictReader(open(path + "/run_counter_collection.csv")):
        e = d.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"],
                                                 "t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return d


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"HIP_vector_type<([a-z ]+), 4u>", r"\1x4", n)
    return n.split("(")[0][:80]


def last_step(d, marker="sgd_flat"):
    ids = list(d)
    marks = [j for j, i in enumerate(ids) if marker in d[i]["name"]]
    return ids[marks[-2] + 1:marks[-1] + 1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sq")
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    A, C, D = load(a.sq), load(a.fetch), load(a.write)
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0.0, 0.0, 0.0, 0])
    for ia, ic, idd in zip(last_step(A), last_step(C), last_step(D)):
        g = agg[short(A[ia]["name"])]
        g[0] += C[ic]["t"]
        g[1] += C[ic].get("FETCH_SIZE", 0.0) * 1024 / 1e9
        g[2] += D[idd].get("WRITE_SIZE", 0.0) * 1024 / 1e9
        g[3] += A[ia].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        g[4] += A[ia]["t"]
        g[5] += 1
    tot = [sum(g[i] for g in agg.values()) for i in range(3)]
    print(f"step: kernel time {tot[0]:.1f} us, read {tot[1]:.2f} GB, written {tot[2]:.2f} GB "
          f"({(tot[1] + tot[2]) / (tot[0] * 1e-6) / 1e3:.2f} TB/s average)")
    print(f"{'us':>8s} {'n':>3s} {'rd GB':>6s} {'wr GB':>6s} {'TB/s':>5s} {'MFMA%':>5s}  kernel")
    for n, g in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        rate = (g[1] + g[2]) / (g[0] * 1e-6) / 1e3 if g[0] else 0.0
        # MFMA busy per SIMD-cycle: 1024 SIMDs at ~2.4 GHz over the SQ pass's own duration
        mf = 100.0 * g[3] / (1024 * 2.4e3 * g[4]) if g[4] else 0.0
        print(f"{g[0]:8.1f} {g[5]:3d} {g[1]:6.2f} {g[2]:6.2f} {rate:5.2f} {mf:5.1f}  {n}")


if __name__ == "__main__":
    main()
