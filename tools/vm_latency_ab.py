"""One zk_vm_prove call alone (vm::prove's shape: host stack pass, states up, trace on the GPU, proof), the benchmark
program at 2^20 with fresh inputs rotating over four sets, timed many times: median and spread for A/B runs of
environment settings (run once per setting, alternating).
    python3 tools/vm_latency_ab.py [calls]      -> one JSON line
"""
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "encrypt-zkvm_amd"):
    sys.path.insert(0, str(p))


def main():
    from zkvm_amd.prover import GpuProver, Program, ProofOptions
    from zkvm_amd.workloads import make_workload, ops_for_trace_len, trace_length
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 31
    src = ops_for_trace_len(20, "cipher")
    prog = Program(src)
    sets = []
    for k in range(4):
        w = make_workload(src, seed=7000 + k)
        sets.append((Program.encode_inputs(w.public, w.secret, w.server_key), w.last_row))
    g = GpuProver(0, max_trace_len=trace_length(src))
    opts = ProofOptions()
    for i in range(5):
        prog.prove_device(g, sets[i % 4][0], sets[i % 4][1], opts)
    ts = []
    for i in range(calls):
        time.sleep(0.01)
        t0 = time.perf_counter()
        prog.prove_device(g, sets[i % 4][0], sets[i % 4][1], opts)
        ts.append(1e3 * (time.perf_counter() - t0))
    g.close()
    ts.sort()
    env = {k: v for k, v in os.environ.items() if k.startswith("ZK_")}
    print(json.dumps({"env": env, "calls": calls, "median_ms": round(statistics.median(ts), 3),
                      "p10_ms": round(ts[len(ts) // 10], 3), "p90_ms": round(ts[(9 * len(ts)) // 10], 3),
                      "min_ms": round(ts[0], 3)}))


if __name__ == "__main__":
    main()
