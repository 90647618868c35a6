"""Soak: many proofs of configs[2]'s program (2^20) on three provers from three host threads, the host-trace path
(`zk_prove_columns`, page-locked traces, whichever upload schedule each proof's company gives it) and `vm::prove`
(`zk_vm_prove`) mixed, over four input sets.  Every proof of an input set must be the same bytes whichever prover and
path made it (the trace and the last row are the same), the seed-1000 set's must equal the oracle pin, and one proof per
set must pass zk_verify.  The provers' hints, the per-device proof count that picks the schedule, the preprocessed-column
cache and the shared upload stream are all exercised under concurrency; nothing may drift over the run.
"""
import hashlib
import threading

import pytest

from golden_large import LARGE_CASES
from zkvm_amd.prover import GpuProver, HostTrace, Program, ProofOptions, make_pub_inputs, verify
from zkvm_amd.workloads import make_workload, ops_for_trace_len

pytestmark = pytest.mark.gpu


def test_mixed_paths_many_proofs():
    c = next(c for c in LARGE_CASES if c["name"] == "c2_cipher_2p20")
    src = ops_for_trace_len(c["log_n"], c["generator"])
    prog = Program(src)
    n = prog.trace_len
    sets, hosts = [], []
    for k, seed in enumerate([c["seed"], 8001, 8002, 8003]):
        w = make_workload(src, seed=seed)
        ht = HostTrace(n)
        hosts.append(ht)
        trace, outputs = prog.trace(w.public, w.secret, w.server_key, w.last_row, out=ht)
        pub = make_pub_inputs(prog.hash, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
        sets.append({"trace": trace, "pub": pub, "inputs": Program.encode_inputs(w.public, w.secret, w.server_key),
                     "last": w.last_row})
    opts = ProofOptions()
    provers = [GpuProver(0, max_trace_len=n) for _ in range(3)]
    got = [dict() for _ in sets]  # set -> {sha256: count}
    errs = []
    lock = threading.Lock()

    def worker(k):
        try:
            for i in range(40):
                s = (i + k) % len(sets)
                if (i + k) % 3 == 2:
                    proof = prog.prove_device(provers[k], sets[s]["inputs"], sets[s]["last"], opts)[2]
                else:
                    proof = provers[k].prove_host(sets[s]["trace"], sets[s]["pub"], opts)[0]
                h = hashlib.sha256(proof).hexdigest()
                with lock:
                    got[s][h] = got[s].get(h, 0) + 1
                    if len(got[s]) == 1 and got[s][h] == 1:
                        sets[s]["proof"] = proof
        except BaseException as e:  # re-raised below
            errs.append(e)

    try:
        ths = [threading.Thread(target=worker, args=(k,)) for k in range(3)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
    finally:
        for g in provers:
            g.close()
        prog.close()
    assert not errs, errs[0]
    assert all(len(d) == 1 for d in got), [list(d.values()) for d in got]  # one proof per input set
    assert sum(sum(d.values()) for d in got) == 120
    assert next(iter(got[0])) == c["proof_sha256"]
    for s in sets:
        assert verify(s["proof"], s["pub"], 95) == (0, "")
    for ht in hosts:
        ht.close()
