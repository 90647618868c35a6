"""Per-kernel time of one loopback sharded proof in the measurement mode (every rank on one stream), for rocprofv3:
python3 tools/shard_kernels.py LOG_N G KIND NPROOFS (KIND device | vm).  Run it under
`rocprofv3 --kernel-trace --stats` twice, with NPROOFS = 1 and 3: the difference of the two summaries / 2 is one
steady-state proof's kernels summed over the G ranks (tools/shard_kernels.py --diff A.csv B.csv G)."""
import csv
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "encrypt-zkvm_amd"))


def run(log_n, G, kind, nproofs):
    from zkvm_amd.prover import Program, ProofOptions, make_pub_inputs, vm_trace
    from zkvm_amd.sharded import ShardedProver
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    src = ops_for_trace_len(log_n, "cipher")
    w = make_workload(src, seed=1000)
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    n = trace.shape[1]
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    prog = Program(src)
    inp = Program.encode_inputs(w.public, w.secret, w.server_key)
    sp = ShardedProver.loopback(G, max_trace_len=n)
    try:
        sp.set_measure(True)
        sp.upload_trace(trace)
        for _ in range(nproofs):
            if kind == "vm":
                sp.prove_program(prog, inp, w.last_row)
            else:
                sp.prove(None, pub, ProofOptions(), n=n)
    finally:
        sp.close()
        prog.close()


def stats(path):
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Name"].split("(")[0].split("<")[0].strip()
            out[name] = out.get(name, 0.0) + float(r["TotalDurationNs"]) / 1e6
            out.setdefault("#" + name, 0)
            out["#" + name] += int(r["Calls"])
    return out


def diff(a, b, G):
    A, B = stats(a), stats(b)
    rows = sorted(((B.get(k, 0) - A.get(k, 0)) / 2, k) for k in B if not k.startswith("#"))
    tot = sum(v for v, _ in rows)
    print(f"one steady-state proof, kernels summed over {G} ranks: {tot:.2f} ms ({tot / G:.2f} per rank)")
    for v, k in reversed(rows):
        if v > 0.01:
            print(f"{k:40s} {v:8.3f} ms  {v / G:7.3f} per rank  launches {(B.get('#' + k, 0) - A.get('#' + k, 0)) / 2:.0f}")


if __name__ == "__main__":
    if sys.argv[1] == "--diff":
        diff(sys.argv[2], sys.argv[3], int(sys.argv[4]))
    else:
        run(int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]))
