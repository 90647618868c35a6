"""Per-kernel wave-cycle breakdown from one rocprofv3 SQ counter pass (where the NTT passes' waves spend their time).

Counters (one pass, 8 SQ): SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, SQ_ACTIVE_INST_VALU,
SQ_ACTIVE_INST_LDS, SQ_WAIT_INST_LDS, SQ_ACTIVE_INST_VMEM.  Per MI355X_MICROARCH.md's PMC table, WAIT_ANY (parked on
s_waitcnt or a barrier) + WAIT_INST_ANY (issue stall) + ACTIVE_INST_ANY (issuing) ~ WAVE_CYCLES, all in quad-cycles;
WAIT_INST_LDS is a sub-bucket of WAIT_INST_ANY.  Kernels are split by template instance (the coset-LDE pass 1 and
the plain one separately).
Usage: python3 tools/pmc_stall.py <rocprofv3 output dir | counter_collection.csv> [-o out.md]
"""
import argparse
import collections
import csv
import glob
import os

COUNTERS = ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
            "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VMEM"]
GROUPS = [("ntt_pass1<10, 4096, true>", "ntt_pass1 CT (coset LDE)"), ("ntt_pass1<10, 4096, false>", "ntt_pass1 plain"),
          ("ntt_pass2", "ntt_pass2"), ("k_eval_constraints", "eval_constraints"), ("k_hash_rows", "hash_rows"),
          ("k_merge", "merkle")]


def group_of(name):
    for key, g in GROUPS:
        if key in name:
            return g
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("-o", default=None)
    args = ap.parse_args()
    path = args.csv
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True))[0]
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = per[r["Dispatch_Id"]]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["name"] = r["Kernel_Name"]
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg = collections.defaultdict(collections.Counter)
    for d in per.values():
        g = group_of(d["name"])
        if g is None or "SQ_WAVE_CYCLES" not in d:
            continue
        a = agg[g]
        a["n"] += 1
        a["ns"] += d["ns"]
        for c in COUNTERS:
            a[c] += d.get(c, 0.0)
    lines = ["| kernel | launches | ms | wait (waitcnt / barrier) | issue stall | of which LDS | issuing | VALU active | "
             "LDS active | VMEM active |", "|---|---|---|---|---|---|---|---|---|---|"]
    for _, g in GROUPS:
        if g not in agg:
            continue
        a = agg[g]
        w = a["SQ_WAVE_CYCLES"] or 1.0
        f = lambda c: f"{a[c] / w:.2f}"
        lines.append(f"| {g} | {a['n']} | {a['ns'] / 1e6:.3f} | {f('SQ_WAIT_ANY')} | {f('SQ_WAIT_INST_ANY')} | "
                     f"{f('SQ_WAIT_INST_LDS')} | {f('SQ_ACTIVE_INST_ANY')} | {f('SQ_ACTIVE_INST_VALU')} | "
                     f"{f('SQ_ACTIVE_INST_LDS')} | {f('SQ_ACTIVE_INST_VMEM')} |")
    out = "\n".join(lines) + "\n\n(fractions of SQ_WAVE_CYCLES, summed over the kernel's launches)\n"
    print(out)
    if args.o:
        open(args.o, "w").write(out)


if __name__ == "__main__":
    main()
