"""Per-proof GPU idle time from a rocprofv3 --kernel-trace CSV of `bench.py` (steady-state proofs).

A proof is delimited by the trace-LDE pass-1 launch with the largest grid (the 8-coset trace LDE);
prints, for the second-to-last complete proof, its span, busy time, idle time and the largest gaps
(with the kernels on either side), plus the number and total time of runtime copy/fill kernels.
Usage: python3 tools/kt_gaps.py <kernel_trace.csv | rocprofv3 output dir>
"""
import csv
import glob
import os
import sys


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    big = max(int(r["Grid_Size_X"]) for r in rows if "ntt_pass1" in r["Kernel_Name"])
    # the proof starts with the trace interpolation, two launches before the big LDE pass 1
    marks = [i - 2 for i, r in enumerate(rows) if "ntt_pass1" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == big]
    if len(marks) < 3:
        sys.exit("fewer than three proofs in the trace")
    a, b = marks[-3], marks[-2]
    p = rows[a:b + 1]
    t0, t1 = int(p[0]["Start_Timestamp"]), int(p[-1]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in p[:-1])
    print(f"kernels {len(p) - 1}  span {(t1 - t0) / 1e3:.0f} us  busy {busy / 1e3:.0f} us  idle {(t1 - t0 - busy) / 1e3:.0f} us")
    gaps = []
    for x, y in zip(p, p[1:]):
        g = (int(y["Start_Timestamp"]) - int(x["End_Timestamp"])) / 1e3
        gaps.append((g, x["Kernel_Name"][:44], y["Kernel_Name"][:44]))
    for g, x, y in sorted(gaps, reverse=True)[:12]:
        print(f"{g:8.1f} us  {x}  ->  {y}")
    rt = [r for r in p[:-1] if r["Kernel_Name"].startswith("__amd_rocclr")]
    print(f"runtime copy/fill kernels: {len(rt)}, {sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in rt) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
