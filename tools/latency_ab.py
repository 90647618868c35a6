"""One prove() call alone from the page-locked host trace (configs[2], the c2_cipher_2p20 pin), timed many times:
median and spread of the single-call latency for A/B runs of environment settings (run once per setting, alternating).
    python3 tools/latency_ab.py [calls]      -> one JSON line
"""
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "encrypt-zkvm_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))


def main():
    from golden_large import LARGE_CASES, large_inputs
    from zkvm_amd.prover import GpuProver
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 31
    c = next(c for c in LARGE_CASES if c["name"] == "c2_cipher_2p20")
    ht, trace, pub, opts = large_inputs(c)
    g = GpuProver(0, max_trace_len=trace.shape[1])
    for _ in range(5):
        g.prove_host(trace, pub, opts)
    ts = []
    for _ in range(calls):
        time.sleep(0.01)
        t0 = time.perf_counter()
        g.prove_host(trace, pub, opts)
        ts.append(1e3 * (time.perf_counter() - t0))
    g.close()
    ht.close()
    ts.sort()
    env = {k: v for k, v in os.environ.items() if k.startswith("ZK_")}
    print(json.dumps({"env": env, "calls": calls, "median_ms": round(statistics.median(ts), 3),
                      "p10_ms": round(ts[len(ts) // 10], 3), "p90_ms": round(ts[(9 * len(ts)) // 10], 3),
                      "min_ms": round(ts[0], 3)}))


if __name__ == "__main__":
    main()
