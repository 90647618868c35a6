"""Summarise one rocprofv3 SQ/GRBM counter pass into a per-kernel VALU-issue table (markdown).

Counters (one pass; see tools/gpu_profile.sh): SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_WAVES, SQ_INSTS_LDS,
SQ_BUSY_CYCLES, SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE, GRBM_COUNT.

  clock      = GRBM_GUI_ACTIVE / n_xcd / kernel duration     (GRBM counts are summed over the 8 XCDs)
  slot_util  = SQ_INSTS_VALU * 2 / (1024 SIMDs * GRBM_GUI_ACTIVE / n_xcd)
               (CDNA4 SIMDs are 32 lanes wide: a plain wave64 VALU instruction issues in 2 cycles;
               measured in tools/ubench/instr*_ubench, profiles/r02_ubench_issue.txt)

slot_util is the fraction of 2-cycle issue slots that carried a VALU instruction.  It cannot reach 1.0
for the f128 kernels: instructions that read or write an SGPR (carry-in/-out, lane-mask selects, the
v_mad_u64_u32 carry-out) issue at most about once per 3.4 cycles per SIMD, and 3-source ops (v_add3,
v_alignbit, v_mad_u64_u32) take two slots, so carry-chain arithmetic saturates near 0.5-0.6 and BLAKE3
near 0.65.  (Round 1 divided by 4-cycle slots and read the same counters as "1.0, instruction bound".)
Usage: python3 tools/pmc_valu.py <counter_collection.csv | rocprofv3 output dir> [-o out.md]
"""
import argparse
import collections
import csv
import glob
import os

GROUPS = [("ntt_pass1", "ntt_pass1"), ("ntt_pass2", "ntt_pass2"), ("ntt_single", "ntt_single"),
          ("k_eval_constraints", "eval_constraints"), ("k_hash_rows", "hash_rows"), ("k_merge", "merkle"),
          ("k_ood", "ood_eval"), ("k_deep", "deep"), ("k_fri", "fri"), ("k_comp_cross", "comp_cross")]
N_XCD = 8
SIMDS = 1024


def group_of(name):
    for key, g in GROUPS:
        if key in name:
            return g
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("-o", default=None)
    ap.add_argument("-j", default=None, help="also write the table as JSON (bench.py reads profiles/pmc_valu.json)")
    args = ap.parse_args()
    path = args.csv
    if os.path.isdir(path):  # rocprofv3 -d DIR: the CSV may sit in a host/pid subdirectory
        path = sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True))[0]
    per = collections.defaultdict(dict)  # dispatch -> counter -> value (+ meta)
    for r in csv.DictReader(open(path)):
        d = per[r["Dispatch_Id"]]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["name"] = r["Kernel_Name"]
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg = collections.defaultdict(lambda: collections.Counter())
    for d in per.values():
        g = group_of(d["name"])
        if g is None or "SQ_INSTS_VALU" not in d:
            continue
        a = agg[g]
        a["n"] += 1
        a["ns"] += d["ns"]
        for k in ("SQ_INSTS_VALU", "GRBM_GUI_ACTIVE", "SQ_WAVES", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_VALU",
                  "SQ_BUSY_CYCLES"):
            a[k] += d.get(k, 0.0)
    lines = ["| kernel | launches | time (ms) | clock (GHz) | VALU instr (G) | slot_util |",
             "|---|---|---|---|---|---|"]
    tot = collections.Counter()
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "encrypt-zkvm_amd"))
    from zkvm_amd.treehash import source_hash
    js = {"source": os.path.abspath(path), "n_xcd": N_XCD, "simds": SIMDS, "tree": source_hash(), "kernels": {}}
    for g, a in sorted(agg.items(), key=lambda kv: -kv[1]["ns"]):
        cyc = a["GRBM_GUI_ACTIVE"] / N_XCD
        issue = a["SQ_INSTS_VALU"] * 2 / (SIMDS * cyc) if cyc else 0.0
        clock = cyc / a["ns"] if a["ns"] else 0.0
        js["kernels"][g] = {"launches": a["n"], "ms": a["ns"] / 1e6, "clock_ghz": clock,
                            "valu_instr": a["SQ_INSTS_VALU"], "slot_util": issue}
        lines.append(f"| {g} | {a['n']} | {a['ns'] / 1e6:.3f} | {clock:.2f} | {a['SQ_INSTS_VALU'] / 1e9:.2f} | "
                     f"{issue:.2f} |")
        tot.update(a)
    cyc = tot["GRBM_GUI_ACTIVE"] / N_XCD
    lines.append(f"| **all above** | {tot['n']} | {tot['ns'] / 1e6:.3f} | {cyc / tot['ns']:.2f} | "
                 f"{tot['SQ_INSTS_VALU'] / 1e9:.2f} | {tot['SQ_INSTS_VALU'] * 2 / (SIMDS * cyc):.2f} |")
    out = "\n".join(lines) + "\n"
    if args.o:
        open(args.o, "w").write(out)
    if args.j:
        import json
        open(args.j, "w").write(json.dumps(js, indent=1) + "\n")
    print(out)


if __name__ == "__main__":
    main()
