"""Idle time between kernels of one steady-state proof, from a rocprofv3 --kernel-trace CSV.

A proof starts at the trace interpolation's first pass (ntt_pass1<.., false> after a non-NTT kernel).
Prints the proof's span, busy time, total gap time and the largest gaps with the kernels around them:
the gaps are the host's share of the critical path (transcript, openings) plus launch latency.
Usage: python3 tools/trace_gaps.py <kernel_trace.csv | rocprofv3 output dir> [which]   (which: -2 = the
second-to-last complete proof, the default)
"""
import csv
import glob
import os
import sys


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
    which = int(sys.argv[2]) if len(sys.argv) > 2 else -2
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    key = "ntt_pass1<10, 4096, false>"
    starts = [i for i, r in enumerate(rows)
              if key in r["Kernel_Name"] and i > 0 and key not in rows[i - 1]["Kernel_Name"]]
    if len(starts) < 2:
        sys.exit("fewer than two proofs in the trace")
    a, b = starts[which - 1], starts[which]
    p = rows[a:b]
    t0, t1 = int(p[0]["Start_Timestamp"]), int(p[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in p)
    print(f"kernels {len(p)}  span {(t1 - t0) / 1e3:.0f} us  busy {busy / 1e3:.0f} us  gaps {(t1 - t0 - busy) / 1e3:.0f} us")
    gaps = []
    for x, y in zip(p, p[1:]):
        g = (int(y["Start_Timestamp"]) - int(x["End_Timestamp"])) / 1e3
        gaps.append((g, x["Kernel_Name"][:40], y["Kernel_Name"][:40]))
    for g, x, y in sorted(gaps, reverse=True)[:20]:
        print(f"{g:8.1f} us  {x}  ->  {y}")
    small = [g for g, _, _ in gaps if g < 5]
    print(f"gaps < 5 us: {len(small)} totalling {sum(small):.0f} us")


if __name__ == "__main__":
    main()
