"""HBM traffic per kernel launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Recipe (/opt/skills/guides/MI355X_MICROARCH.md, "HBM" and "rocprofv3 PMC slots"):
  * FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950 -> two separate runs;
  * both are reported in KiB;
  * on gfx950 FETCH_SIZE counts exactly half the bytes of wide coalesced streaming reads ->
    doubled here; WRITE_SIZE is exact for 16-B-per-lane streaming stores.
The traffic of a launch = 2 * FETCH_SIZE + WRITE_SIZE (bytes), averaged over all dispatches
of a kernel.  Kernel names are mapped onto the in-library profiler names bench.py reports.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> [-o profiles/pmc_traffic.json]
"""
from __future__ import annotations

import argparse
import csv
import json
import re
from collections import defaultdict
from pathlib import Path

ALIASES = {"k_merge_level": "merkle_level", "k_merge_top": "merkle_top", "k_batch_inv_pairs": "batch_inv"}


def short_name(kernel: str) -> str:
    k = re.sub(r"^void\s+", "", kernel)
    k = k.split("(")[0].split("<")[0]
    k = k.split("::")[-1]
    if k in ALIASES:
        return ALIASES[k]
    return k[2:] if k.startswith("k_") else k


def read_counter(d: Path, counter: str):
    """-> {kernel: [value per dispatch]} summed over counter instances of a dispatch."""
    files = sorted(d.rglob("*counter_collection.csv"))
    if not files:
        raise SystemExit(f"no *counter_collection.csv under {d}")
    per = defaultdict(lambda: defaultdict(float))
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                per[short_name(row["Kernel_Name"])][(f.name, row.get("Dispatch_Id"))] += float(row["Counter_Value"])
    return {k: list(v.values()) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("-o", "--out", default="profiles/pmc_traffic.json")
    a = ap.parse_args()
    fetch = read_counter(Path(a.fetch_dir), "FETCH_SIZE")
    write = read_counter(Path(a.write_dir), "WRITE_SIZE")
    out = {"method": "per launch: (2 x FETCH_SIZE + WRITE_SIZE) x 1024 B, averaged over dispatches; FETCH_SIZE "
                     "doubled per the gfx950 correction in MI355X_MICROARCH.md; separate --pmc passes",
           "per_launch_bytes": {}, "fetch_kib_avg": {}, "write_kib_avg": {}, "dispatches": {}}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        if not f or not w:
            continue
        fa, wa = sum(f) / len(f), sum(w) / len(w)
        out["fetch_kib_avg"][k] = round(fa, 1)
        out["write_kib_avg"][k] = round(wa, 1)
        out["per_launch_bytes"][k] = round((2 * fa + wa) * 1024)
        out["dispatches"][k] = len(f)
    Path(a.out).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out["per_launch_bytes"], indent=1))


if __name__ == "__main__":
    main()
