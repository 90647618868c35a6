"""The lead-only window of one loopback sharded proof (tools/shard_kernels.py under rocprofv3 --kernel-trace): from
the last proof's layer-1 permute (the first kernel after the FRI layer-1 all-gather) to its first openings gather,
the kernels in it and the device idle between them.  python3 tools/lead_window.py KERNEL_TRACE.csv"""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
starts = [i for i, r in enumerate(rows) if "k_sh_permute" in r[2]]
i0 = starts[-1]
i1 = next(i for i in range(i0, len(rows)) if "gather_chunks" in rows[i][2])
win = rows[i0:i1]
busy = sum(e - s for s, e, _ in win)
span = rows[i1][0] - rows[i0][0]
print(f"lead window: {span / 1e6:.3f} ms, kernels {busy / 1e6:.3f} ms in {len(win)} launches, idle {(span - busy) / 1e6:.3f} ms")
agg = {}
for s, e, k in win:
    name = k.split("(")[0].replace("void ", "")[-48:]
    agg.setdefault(name, [0, 0])
    agg[name][0] += e - s
    agg[name][1] += 1
for k, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0]):
    print(f"  {t / 1e6:7.3f} ms {c:4d}  {k}")
gaps = sorted(((rows[i + 1][0] - rows[i][1]), rows[i][2][:40], rows[i + 1][2][:40]) for i in range(i0, i1))[-6:]
for g, a, b in reversed(gaps):
    print(f"  gap {g / 1e6:.3f} ms after {a} before {b}")
