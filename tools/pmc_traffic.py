"""HBM traffic per kernel launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Recipe (/opt/skills/guides/MI355X_MICROARCH.md, "HBM" and "rocprofv3 PMC slots"):
  * FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950 -> two separate runs;
  * both are reported in KiB;
  * on gfx950 FETCH_SIZE counts exactly half the bytes of wide coalesced streaming reads ->
    doubled here; WRITE_SIZE is exact for 16-B-per-lane streaming stores.
The traffic of a launch = 2 * FETCH_SIZE + WRITE_SIZE (bytes).  Kernel names are mapped onto the in-library
profiler names bench.py reports.  With --bench (the bench line the FETCH pass printed: one prover, warm-up proofs
first, so its last proof is a steady-state, hinted one) the figures are the LAST proof's: per kernel, the last
`kernel_launches[k]` dispatches (the launches one proof makes), summed per proof and per launch, against that
proof's algorithmic bytes (`kernel_alg_bytes`) -> traffic_ratio.  The output is stamped with the source hash of the
tree it ran on (zkvm_amd.treehash).

    python tools/pmc_traffic.py <fetch_dir> <write_dir> [--bench fetch_bench.json] [-o profiles/pmc_traffic.json]
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "encrypt-zkvm_amd"))

ALIASES = {"k_merge_level": "merkle_level", "k_merge_top": "merkle_top", "k_batch_inv_pairs": "batch_inv",
           "k_hash_rows_blocks": "hash_rows"}  # (the library profiler counts both row-hashing kernels as hash_rows)


def short_name(kernel: str) -> str:
    k = re.sub(r"^void\s+", "", kernel)
    k = k.split("(")[0].split("<")[0]
    k = k.split("::")[-1]
    if k in ALIASES:
        return ALIASES[k]
    return k[2:] if k.startswith("k_") else k


def read_counter(d: Path, counter: str):
    """-> {kernel: [value per dispatch, in dispatch order]} summed over counter instances of a dispatch."""
    files = sorted(d.rglob("*counter_collection.csv"))
    if not files:
        raise SystemExit(f"no *counter_collection.csv under {d}")
    per = defaultdict(lambda: defaultdict(float))
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                did = row.get("Dispatch_Id") or "0"
                per[short_name(row["Kernel_Name"])][(f.name, int(did) if did.isdigit() else did)] += float(row["Counter_Value"])
    return {k: [v[key] for key in sorted(v)] for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--bench", help="the bench JSON line of the FETCH pass (kernel_launches, kernel_alg_bytes)")
    ap.add_argument("-o", "--out", default="profiles/pmc_traffic.json")
    a = ap.parse_args()
    from zkvm_amd.treehash import source_hash
    fetch = read_counter(Path(a.fetch_dir), "FETCH_SIZE")
    write = read_counter(Path(a.write_dir), "WRITE_SIZE")
    bench = None
    if a.bench:
        bench = json.loads(Path(a.bench).read_text().strip().splitlines()[-1])
    launches = (bench or {}).get("kernel_launches", {})
    alg = (bench or {}).get("kernel_alg_bytes", {})
    out = {"method": "(2 x FETCH_SIZE + WRITE_SIZE) x 1024 B per dispatch (FETCH_SIZE doubled per the gfx950 correction "
                     "in MI355X_MICROARCH.md; separate --pmc passes); with launches per proof known, the last proof's "
                     "dispatches only (steady state, hints in use)",
           "tree": source_hash(), "scope": "last proof" if launches else "all dispatches",
           "per_launch_bytes": {}, "per_proof_bytes": {}, "alg_per_proof_bytes": {}, "traffic_ratio": {},
           "launches_per_proof": {}, "fetch_kib_avg": {}, "write_kib_avg": {}, "dispatches": {}}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        if not f or not w:
            continue
        L = launches.get(k)
        if L and L <= min(len(f), len(w)):
            f, w = f[-L:], w[-L:]
            tot = round((2 * sum(f) + sum(w)) * 1024)
            out["per_proof_bytes"][k] = tot
            out["launches_per_proof"][k] = L
            if alg.get(k):
                out["alg_per_proof_bytes"][k] = round(alg[k])
                out["traffic_ratio"][k] = round(tot / alg[k], 4)
        fa, wa = sum(f) / len(f), sum(w) / len(w)
        out["fetch_kib_avg"][k] = round(fa, 1)
        out["write_kib_avg"][k] = round(wa, 1)
        out["per_launch_bytes"][k] = round((2 * fa + wa) * 1024)
        out["dispatches"][k] = len(f)
    Path(a.out).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps({"tree": out["tree"], "traffic_ratio": out["traffic_ratio"]}, indent=1))


if __name__ == "__main__":
    main()
