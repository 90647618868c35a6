"""Wall time of every proof in a loop of 2^20 proofs on one GPU (one prover), to find outliers.
Usage (GPU box): python3 tools/proof_times.py [count]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "encrypt-zkvm_amd"))

from zkvm_amd.prover import GpuProver, ProofOptions, make_pub_inputs, vm_trace  # noqa: E402
from zkvm_amd.workloads import make_workload, ops_for_trace_len  # noqa: E402


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    src = ops_for_trace_len(20, "cipher")
    w = make_workload(src, seed=1000)
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    n = trace.shape[1]
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    g = GpuProver(0, max_trace_len=n)
    d = g.upload_trace(trace)[0]
    ts = []
    for _ in range(count):
        t0 = time.perf_counter()
        g.prove_device(d, n, pub, ProofOptions())
        ts.append(1e3 * (time.perf_counter() - t0))
    print(" ".join(f"{t:.2f}" for t in ts))
    s = sorted(ts[2:])
    print(f"median {s[len(s) // 2]:.3f} ms  min {s[0]:.3f}  max {s[-1]:.3f}  mean {sum(s) / len(s):.3f}")
    g.close()


if __name__ == "__main__":
    main()
