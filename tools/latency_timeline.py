"""One prove() call alone, as a timeline: kernels and copies of the call from a rocprofv3 trace.

Run (GPU box):
  cd /tmp && rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/lat -o lat -- \
      python3 $R/tools/latency_timeline.py --out $R/gpurun_out/lat_marks.json
  python3 $R/tools/latency_timeline.py --analyze $R/gpurun_out/lat --marks $R/gpurun_out/lat_marks.json
The run part proves the configs[2] trace (2^20, seed 1000, page-locked; --vm: the same program and inputs through
zk_vm_prove) with one prover: 5 warm-up calls, then 3
timed calls 100 ms apart, each bracketed by CLOCK_MONOTONIC stamps (the clock rocprofv3's timestamps use).  The
analysis takes the last timed call and reports: call start -> first copy, -> first kernel; the last copy's end; the
device-idle gaps between kernels (host round trips of the transcript) with the kernel after each; busy time; and the
tail from the last kernel's end to the call's return.
"""
import argparse
import csv
import glob
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "encrypt-zkvm_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))


def run(out, vm=False):
    from golden_large import LARGE_CASES, large_inputs
    from zkvm_amd.prover import GpuProver, Program, ProofOptions
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    c = next(c for c in LARGE_CASES if c["name"] == "c2_cipher_2p20")
    if vm:  # zk_vm_prove: the same program and inputs, the trace written on the GPU
        src = ops_for_trace_len(c["log_n"], c["generator"])
        w = make_workload(src, seed=c["seed"])
        prog = Program(src)
        inputs = Program.encode_inputs(w.public, w.secret, w.server_key)
        g = GpuProver(0, max_trace_len=prog.trace_len)
        call = lambda: prog.prove_device(g, inputs, w.last_row, ProofOptions())  # noqa: E731
        ht = None
    else:
        ht, trace, pub, opts = large_inputs(c)
        g = GpuProver(0, max_trace_len=trace.shape[1])
        call = lambda: g.prove_host(trace, pub, opts)  # noqa: E731
    for _ in range(5):
        call()
    marks = []
    for _ in range(3):
        time.sleep(0.1)
        t0 = time.monotonic_ns()
        call()
        t1 = time.monotonic_ns()
        marks.append((t0, t1))
    g.close()
    if ht:
        ht.close()
    Path(out).write_text(json.dumps({"calls": marks}))
    print("calls (ms):", [round((b - a) / 1e6, 3) for a, b in marks])


def rows(d, pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def analyze(d, marks_file):
    t0, t1 = json.loads(Path(marks_file).read_text())["calls"][-1]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "?")) for r in rows(d, "*kernel_trace.csv")]
    cs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "?"), r.get("Bytes") or r.get("Size") or "?")
          for r in rows(d, "*memory_copy_trace.csv")]
    if not any(t0 <= k[0] <= t1 for k in ks):
        # the profiler's clock is not CLOCK_MONOTONIC here: take the last burst of activity (the calls are 100 ms
        # apart) and anchor the call's start at its first copy (the call's first device action)
        ev = sorted([(k[0], k[1]) for k in ks] + [(c[0], c[1]) for c in cs])
        start = ev[-1][0]
        for (s0, e0), (s1, _) in zip(reversed(ev[:-1]), reversed(ev[1:])):
            if s1 - e0 > 50_000_000:
                break
            start = s0
        dur = t1 - t0
        t0, t1 = start, start + dur
        print("(profiler clock differs: the call is anchored at its first device event)")
    ks = sorted(k for k in ks if t0 <= k[0] <= t1)
    cs = sorted(c for c in cs if t0 <= c[0] <= t1)
    ms = lambda x: round(x / 1e6, 3)  # noqa: E731
    busy, gaps, end = 0, [], None
    for s, e, name in ks:
        if end is not None and s > end:
            gaps.append((s - end, name.split("(")[0][-60:]))
        end = e if end is None else max(end, e)
        busy += e - s
    h2d = [c for c in cs if "HOST_TO_DEVICE" in c[2].upper() or "H2D" in c[2].upper()]
    rep = {
        "call_ms": ms(t1 - t0),
        "first_copy_start_ms": ms(cs[0][0] - t0) if cs else None,
        "first_h2d_end_ms": ms(h2d[0][1] - t0) if h2d else None,
        "first_kernel_start_ms": ms(ks[0][0] - t0) if ks else None,
        "last_h2d_end_ms": ms(max(c[1] for c in h2d) - t0) if h2d else None,
        "last_kernel_end_ms": ms(end - t0) if end else None,
        "tail_after_last_kernel_ms": ms(t1 - end) if end else None,
        "kernel_busy_ms": ms(busy), "kernels": len(ks), "copies": len(cs), "h2d_copies": len(h2d),
        "idle_gaps_total_ms": ms(sum(g for g, _ in gaps)),
        "largest_gaps": [{"ms": ms(g), "before": n} for g, n in sorted(gaps, reverse=True)[:12]],
    }
    print(json.dumps(rep, indent=1))
    return rep


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--analyze")
    ap.add_argument("--marks")
    ap.add_argument("--vm", action="store_true", help="time zk_vm_prove (vm::prove's shape) instead of prove_host")
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze, a.marks)
    else:
        run(a.out, a.vm)
