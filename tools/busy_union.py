"""Device occupancy of a multi-prover run from a rocprofv3 --kernel-trace CSV: over the middle of the run (kernels
between the 30 % and 80 % marks by start time, i.e. steady state with P provers in flight), the union of the kernel
intervals against the wall time (1 - idle fraction) and the summed kernel time over that union (how many kernels run
at once on average).  Usage: python3 tools/busy_union.py <kernel_trace.csv | rocprofv3 output dir>
"""
import csv
import glob
import os
import sys


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(path)))
    a, b = ks[int(0.3 * len(ks))][0], ks[int(0.8 * len(ks))][0]
    sel = [(max(s, a), min(e, b)) for s, e in ks if e > a and s < b]
    busy, cur_s, cur_e, tot = 0, None, None, 0
    for s, e in sel:
        tot += e - s
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = b - a
    print(f"window {wall / 1e6:.1f} ms, kernels {len(sel)}, busy (union) {busy / wall:.4f}, idle {1 - busy / wall:.4f}, "
          f"mean concurrency {tot / busy:.2f}")


if __name__ == "__main__":
    main()
