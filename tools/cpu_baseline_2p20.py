"""The CPU baseline on the headline config itself (the bench's cpu_baseline samples 2^18 so that a
default run stays within minutes): the oracle's single-threaded or_prove on configs[2]'s own 2^20 trace (the
c2_cipher_2p20 pin's workload: cipher mix, seed 1000, reference options), timed on this host, its proof checked
against the pin.  Oracle = test infrastructure, used here only as the CPU reference prover being timed.
    python3 tools/cpu_baseline_2p20.py [runs]     (prints one JSON object)
"""
import hashlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "encrypt-zkvm_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))

from golden_large import LARGE_CASES, oracle_pub  # noqa: E402
from oracle import oracle  # noqa: E402
from zkvm_amd.prover import make_pub_inputs, vm_trace  # noqa: E402
from zkvm_amd.workloads import make_workload, ops_for_trace_len  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    c = next(c for c in LARGE_CASES if c["name"] == "c2_cipher_2p20")
    src = ops_for_trace_len(c["log_n"], c["generator"])
    w = make_workload(src, seed=c["seed"])
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    assert hashlib.sha256(trace.tobytes()).hexdigest() == c["trace_sha256"]
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    oracle.build()
    n = trace.shape[1]
    times = []
    for _ in range(runs):
        t0 = time.perf_counter()
        proof, _, _ = oracle.prove(trace, oracle_pub(oracle, pub))
        times.append(time.perf_counter() - t0)
        assert hashlib.sha256(proof).hexdigest() == c["proof_sha256"], "oracle proof differs from the pin"
    med = sorted(times)[len(times) // 2]
    print(json.dumps({"config": "configs[2] (c2_cipher_2p20: 2^20 cipher mix, seed 1000, reference options)",
                      "kind": "port", "cores": 1, "runs_s": [round(t, 2) for t in times], "median_s": round(med, 2),
                      "trace_steps_per_s": round(n / med, 1), "proof_matches_pin": True,
                      "host_cpus": os.cpu_count()}))


if __name__ == "__main__":
    main()
