"""Throughput of independent 2^20 proofs on ONE GPU: one prover in a loop vs P provers (own buffers,
own streams) driven by P host threads, so one prover's host round trips and its proof tail overlap the
other provers' kernels.  Usage (GPU box): python3 tools/dual_prover.py [steps] [provers...]
"""
import os
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "encrypt-zkvm_amd"))

from zkvm_amd.prover import GpuProver, ProofOptions, make_pub_inputs, vm_trace  # noqa: E402
from zkvm_amd.workloads import make_workload, ops_for_trace_len  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    counts = [int(a) for a in sys.argv[2:]] or [1, 2, 3]
    src = ops_for_trace_len(20, "cipher")
    w = make_workload(src, seed=1000)
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    n = trace.shape[1]
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    opts = ProofOptions()
    provers = [GpuProver(0, max_trace_len=n) for _ in range(max(counts))]
    dts = [g.upload_trace(trace)[0] for g in provers]
    ref = provers[0].prove_device(dts[0], n, pub, opts)[0]
    for g, d in zip(provers, dts):
        assert g.prove_device(d, n, pub, opts)[0] == ref
    for P in counts * 2:
        per = steps // P
        out = [None] * P

        def run(k):
            g, d = provers[k], dts[k]
            for _ in range(per):
                out[k] = g.prove_device(d, n, pub, opts)[0]

        ths = [threading.Thread(target=run, args=(k,)) for k in range(P)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        dt = time.perf_counter() - t0
        assert all(o == ref for o in out)
        print(f"provers={P} proofs={per * P} {1e3 * dt / (per * P):.3f} ms/proof "
              f"{n * per * P / dt / 1e6:.1f} M trace-steps/s", flush=True)
    for g in provers:
        g.close()


if __name__ == "__main__":
    main()
