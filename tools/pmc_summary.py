"""Per-dispatch PMC table for one training step from rocprofv3 --pmc CSVs (scripts/gpu_profile.sh (PMC=1)).

    python tools/pmc_summary.py gpurun_out/pmcA/run_counter_collection.csv \
        [gpurun_out/pmcB/run_counter_collection.csv] [--step -1] [--marker sgd_flat]

Columns: duration, MFMA utilisation (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel cycles), kernel
cycles = GRBM_GUI_ACTIVE / 8 XCDs from the second pass, else duration x 2.1 GHz; never more than
duration x 2.4 GHz, MI355X's peak engine clock -- GRBM_GUI_ACTIVE of a short dispatch also counts the
busy cycles around it, and such rows are marked '*' in the GHz column), and the wave-state
split of SQ_WAVE_CYCLES: parked (SQ_WAIT_ANY: s_waitcnt / barrier), issue-stalled
(SQ_WAIT_INST_ANY), issuing (SQ_ACTIVE_INST_ANY); LDS-issue stalls and bank-conflict cycles per wave
cycle.  Passes are matched by dispatch id (the step's launch sequence is deterministic).
"""
import argparse
import collections
import csv

PEAK_GHZ = 2.4  # MI355X peak engine clock: no dispatch runs more cycles than duration x this


def load(path):
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                                                     "wg": int(r["Workgroup_Size"]),
                                                     "t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"]),
                                                     "vgpr": r["VGPR_Count"], "agpr": r["Accum_VGPR_Count"],
                                                     "lds": r["LDS_Block_Size"]})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return disp


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = name[5:] if name.startswith("void ") else name
    return name.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b", nargs="?")
    ap.add_argument("--step", type=int, default=-1)
    ap.add_argument("--marker", default="sgd_flat")
    a = ap.parse_args()
    A = load(a.a)
    B = load(a.b) if a.b else {}
    ids = list(A)
    marks = [i for i, d in enumerate(ids) if a.marker in A[d]["name"]]
    lo = marks[a.step - 1] + 1 if len(marks) >= 2 else 0
    hi = marks[a.step] + 1
    print(f"{'dur_us':>7} {'mfma%':>6} {'park%':>6} {'stall%':>6} {'issue%':>6} {'ldsst%':>6} {'bank%':>6} "
          f"{'GHz':>5} {'vgpr':>4} {'agpr':>4} {'lds':>6} {'wgs':>6}  kernel")
    tot = collections.defaultdict(float)
    for d in ids[lo:hi]:
        r = A[d]
        dur = (r["t1"] - r["t0"]) / 1e3
        rb = B.get(d, {})
        cyc = rb.get("GRBM_GUI_ACTIVE", 0.0) / 8 if rb else dur * 1e3 * 2.1
        clamped = cyc > dur * 1e3 * PEAK_GHZ
        if clamped:
            cyc = dur * 1e3 * PEAK_GHZ
        ghz = cyc / (dur * 1e3) if dur > 0 else 0.0
        mf = r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * cyc) * 100 if cyc else 0.0
        wc = r.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        pk = r.get("SQ_WAIT_ANY", 0.0) / wc * 100
        st = r.get("SQ_WAIT_INST_ANY", 0.0) / wc * 100
        iss = r.get("SQ_ACTIVE_INST_ANY", 0.0) / wc * 100
        ls = r.get("SQ_WAIT_INST_LDS", 0.0) / wc * 100
        bc = r.get("SQ_LDS_BANK_CONFLICT", 0.0) / wc * 100
        nwg = r["grid"] // max(r["wg"], 1)
        print(f"{dur:7.1f} {mf:6.1f} {pk:6.1f} {st:6.1f} {iss:6.1f} {ls:6.1f} {bc:6.1f} {ghz:4.2f}{'*' if clamped else ' '} {r['vgpr']:>4} "
              f"{r['agpr']:>4} {r['lds']:>6} {nwg:6d}  {short(r['name'])}")
        tot["dur"] += dur
        tot["mfma_cyc"] += r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        tot["cyc"] += cyc
    print(f"step kernel time {tot['dur']:.1f} us, MFMA utilisation over the step "
          f"{tot['mfma_cyc'] / (1024 * tot['cyc']) * 100 if tot['cyc'] else 0:.1f} %")


if __name__ == "__main__":
    main()
