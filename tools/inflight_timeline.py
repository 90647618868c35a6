"""Timeline of the bench's timed region: P provers in flight, host-resident (page-locked) 2^20 trace, K proofs dealt
round-robin as bench.py does, every proof's start / end relative to the region's start.  Shows where a short run
loses against the steady state (fill at the start, drain at the end, lockstep phases in between).
Usage (GPU box, repo root):  python3 tools/inflight_timeline.py [K=20] [P=4] [reps=3]"""
import os
import sys
import threading
import time
from pathlib import Path

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "encrypt-zkvm_amd"))

from zkvm_amd.prover import GpuProver, HostTrace, Program, ProofOptions, make_pub_inputs  # noqa: E402
from zkvm_amd.workloads import make_workload, ops_for_trace_len, trace_length  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    src = ops_for_trace_len(20, "cipher")
    w = make_workload(src, seed=1000)
    n = trace_length(src)
    host = HostTrace(n)
    prog = Program(src)
    trace, outputs = prog.trace(w.public, w.secret, w.server_key, w.last_row, out=host)
    pub = make_pub_inputs(prog.hash, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    prog.close()
    provers = [GpuProver(0, max_trace_len=n) for _ in range(P)]
    opts = ProofOptions()

    def run(count, log):
        share = [count // P + (1 if k < count % P else 0) for k in range(P)]
        t0 = time.perf_counter()

        def body(k):
            for _ in range(share[k]):
                a = time.perf_counter()
                provers[k].prove_host(trace, pub, opts)
                log.append((k, 1e3 * (a - t0), 1e3 * (time.perf_counter() - t0)))

        ths = [threading.Thread(target=body, args=(k,)) for k in range(P) if share[k]]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        return 1e3 * (time.perf_counter() - t0)

    run(3 * P, [])  # warm-up
    for r in range(reps):
        log = []
        total = run(K, log)
        log.sort(key=lambda x: x[2])
        print(f"rep {r}: {K} proofs, {P} in flight: {total:.1f} ms = {total / K:.3f} ms per proof")
        ends = [e for _, _, e in log]
        gaps = [b - a for a, b in zip([0.0] + ends[:-1], ends)]
        print("  completions (ms): " + " ".join(f"{e:.1f}" for e in ends))
        print("  inter-completion: " + " ".join(f"{g:.1f}" for g in gaps))
        lat = sorted(e - s for _, s, e in log)
        print(f"  proof latency: min {lat[0]:.1f} median {lat[len(lat) // 2]:.1f} max {lat[-1]:.1f}")
    for g in provers:
        g.close()
    host.close()


if __name__ == "__main__":
    main()
