"""One rank of a multi-process coset-sharded proof (zk_prove_sharded over zk_comm_create_host + a TCP host group).

Started by tests/test_sharded_multiprocess.py, `world` copies at once, all on GPU 0 of the test box: every process
holds one rank-sized prover and exchanges through zkvm_amd.hostgroup (TCP over 127.0.0.1; torch-free, so the library
runs on the HIP runtime it links), which is the code path an RCCL rank runs (one local rank per process, rank-dependent ownership of cosets, openings and FRI layers) with the
transport swapped.  Each job's proof sha256 goes to <out>/rank<r>.json; the test compares them with the golden
proofs and, for the generated traces, with the single-GPU prover's proof (computed on rank 0).

usage: python tests/sharded_worker.py RANK WORLD PORT OUTDIR [selftest | large:<pinned case>]
"""
import hashlib
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "encrypt-zkvm_amd"):
    sys.path.insert(0, str(p))

import numpy as np  # noqa: E402

GOLD = ROOT / "tests" / "golden"


def golden_jobs(world):
    from zkvm_amd.prover import ProofOptions, make_pub_inputs
    jobs = []
    for c in json.loads((GOLD / "cases.json").read_text())["cases"]:
        o = c["options"]
        n, fold = c["trace_len"], o["fri_folding"]
        if o["blowup"] != 8 or n // fold < 8 * world or n // world < 8:
            continue
        trace = np.load(GOLD / f"{c['name']}.trace.npy", allow_pickle=False)
        pub = make_pub_inputs([int(h, 16) for h in c["program_hash"]], [int(h, 16) for h in c["stack_outputs"]],
                              c["lwe_size"], c["delta"])
        opts = ProofOptions(o["num_queries"], o["blowup"], o["grinding"], o["field_extension"], fold,
                            o["fri_rem_max_deg"])
        want = hashlib.sha256((GOLD / f"{c['name']}.proof").read_bytes()).hexdigest()
        jobs.append((c["name"], trace, pub, opts, want))
    return jobs


def generated_jobs(rank):
    """VM traces of the cipher-mix workload; the expected hash is the single-GPU prover's (rank 0 computes it)."""
    from zkvm_amd.prover import GpuProver, ProofOptions, make_pub_inputs, vm_trace
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    jobs = []
    for log_n, ext in ((16, 1), (14, 2)):
        src = ops_for_trace_len(log_n, "cipher")
        w = make_workload(src, seed=31 + log_n)
        trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
        pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
        opts = ProofOptions(field_extension=ext)
        want = None
        if rank == 0:
            g = GpuProver(0, max_trace_len=trace.shape[1])
            try:
                single, _, _, rc = g.prove(trace, pub, opts)
                assert rc == 0
                want = hashlib.sha256(single).hexdigest()
            finally:
                g.close()
        jobs.append((f"cipher_2p{log_n}_ext{ext}", trace, pub, opts, want))
    return jobs


def selftest(rank, world, fn):
    """The exchange callback alone (no GPU): both ops through the C calling convention, chunk order checked."""
    import ctypes as C
    from zkvm_amd import native
    nb = 5
    send = (C.c_uint8 * (nb * world))(*[(16 * rank + d) & 255 for d in range(world) for _ in range(nb)])
    recv = (C.c_uint8 * (nb * world))()
    assert fn(None, native.XCHG_ALL_TO_ALL, C.addressof(send), C.addressof(recv), nb) == 0
    a2a = list(recv)
    one = (C.c_uint8 * nb)(*[rank + 100] * nb)
    assert fn(None, native.XCHG_ALL_GATHER, C.addressof(one), C.addressof(recv), nb) == 0
    ag = list(recv)
    bad = fn(None, 7, C.addressof(one), C.addressof(recv), nb)
    return {"a2a": a2a, "ag": ag, "bad_op_rc": bad}


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], Path(sys.argv[4])
    mode = sys.argv[5] if len(sys.argv) > 5 else "prove"
    from zkvm_amd.hostgroup import HostGroup
    from zkvm_amd.sharded import ShardedProver
    dist = HostGroup(rank, world, port=int(port), timeout=120)
    fn = dist.exchange_fn()
    if mode == "selftest":
        (out / f"rank{rank}.json").write_text(json.dumps(selftest(rank, world, fn)))
        dist.close()
        return
    if mode.startswith("large:"):  # one full-size pinned case (tests/golden/large), checked here on every rank
        sys.path.insert(0, str(ROOT / "tests"))
        from golden_large import LARGE_CASES, check_large_proof, large_inputs
        from oracle import oracle
        c = next(c for c in LARGE_CASES if c["name"] == mode[len("large:"):])
        ht, trace, pub, opts = large_inputs(c)
        sp = ShardedProver.host(rank, world, fn, 0, trace.shape[1])
        try:
            proof, rec = sp.prove(trace, pub, opts, record=True)
        finally:
            sp.close()
            ht.close()
        check_large_proof(c, proof, rec, pub, oracle)  # the parent test built the oracle library
        (out / f"rank{rank}.json").write_text(json.dumps({c["name"]: {"sha256": hashlib.sha256(proof).hexdigest(),
                                                                       "want": c["proof_sha256"]}}))
        dist.close()
        return
    jobs = golden_jobs(world) + generated_jobs(rank)
    res = {}
    sp = ShardedProver.host(rank, world, fn, 0, max(t.shape[1] for _, t, _, _, _ in jobs))
    try:
        for name, trace, pub, opts, want in jobs:
            proof, _ = sp.prove(trace, pub, opts)
            res[name] = {"sha256": hashlib.sha256(proof).hexdigest(), "want": want, "bytes": len(proof)}
            print(f"rank {rank}/{world} {name}: {len(proof)} B", flush=True)
        # vm::prove sharded (zk_vm_prove_sharded): this rank writes the 2^16 job's trace into its own HBM and builds the
        # preprocessed columns of its own cosets; the proof must equal the host-trace job's
        from zkvm_amd.prover import Program, ProofOptions
        from zkvm_amd.workloads import make_workload, ops_for_trace_len
        src = ops_for_trace_len(16, "cipher")
        w = make_workload(src, seed=31 + 16)
        prog = Program(src)
        try:
            for k in range(2):  # the second call reuses the rank's preprocessed columns
                _, _, proof = sp.prove_program(prog, Program.encode_inputs(w.public, w.secret, w.server_key),
                                               w.last_row, ProofOptions())
                res[f"vm_cipher_2p16_call{k}"] = {"sha256": hashlib.sha256(proof).hexdigest(),
                                                  "want": res["cipher_2p16_ext1"]["want"], "bytes": len(proof)}
        finally:
            prog.close()
    finally:
        sp.close()
    from zkvm_amd import native
    res["runtime"] = native.runtime_info()
    (out / f"rank{rank}.json").write_text(json.dumps(res))
    dist.close()


if __name__ == "__main__":
    main()
