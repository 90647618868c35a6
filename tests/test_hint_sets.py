"""Column hints keyed by (trace length, program hash) (prover.hip hint_find / hint_slot).

A host-resident trace's column classes -- sparse (zero but the last row), narrow (8- / 32-bit before the last row),
the AIR clock -- are learned from one proof and used by the next proof of the same length AND program, so a server
that alternates programs of one length keeps each program's hints instead of voiding the other's proofs (a refuted
hint costs a redone proof).  Here two programs of one trace length with different sparse sets alternate on one
prover: the cipher mix (stack registers s11..s15 stay zero) and push/add (s2..s15 stay zero).  Under the round-5
length-only key, push/add's hints (columns 14..27 sparse) were refuted by every following cipher-mix proof.
"""
import pytest

from test_gpu_parity import oracle_pub, workload_trace
from zkvm_amd.prover import GpuProver, ProofOptions
from zkvm_amd.workloads import ops_for_trace_len

pytestmark = pytest.mark.gpu


def test_alternating_programs_keep_their_own_hints(oracle):
    ta, pa = workload_trace(ops_for_trace_len(14, "cipher"), seed=21)
    tb, pb = workload_trace(ops_for_trace_len(14, "pushadd"), seed=22)
    assert ta.shape == tb.shape and bytes(pa.program_hash) != bytes(pb.program_hash)
    n = ta.shape[1]
    want = {k: oracle.prove(t, oracle_pub(oracle, p))[0] for k, (t, p) in (("a", (ta, pa)), ("b", (tb, pb)))}
    g = GpuProver(0, max_trace_len=n)
    try:
        seen = {"a": [], "b": []}
        for k in "ababab":
            t, p = (ta, pa) if k == "a" else (tb, pb)
            proof, _, _, rc = g.prove(t, p, ProofOptions())
            assert rc == 0 and proof == want[k], k
            seen[k].append((g.proof_info(), g.upload_stats()))
        info = g.proof_info()
        assert info["hint_redos"] == 0, info  # no proof was voided by the other program's hints
        assert info["hint_sets"] == 2
        # from each program's second proof on: its own sparse columns hinted (never uploaded), the clock derived
        sparse = {k: [c for c in range(28) if not t[c, : n - 1].any()] for k, t in (("a", ta), ("b", tb))}
        assert sparse["a"] == list(range(23, 28)) and set(range(14, 28)) <= set(sparse["b"])
        for k, cols in sparse.items():
            for pi, up in seen[k][1:]:
                assert pi["hinted_sparse"] == cols, (k, pi)
                assert up["sparse"] == cols and up["derived"] == [0], (k, up)
    finally:
        g.close()


def test_hint_sets_evict_least_recently_used(oracle):
    """More programs than hint sets (8): the least recently used set is evicted, every proof stays the oracle's."""
    progs = []
    for k in range(10):
        src = ops_for_trace_len(13, "cipher" if k % 2 else "pushadd")
        src = src + f"\npush.{k + 1}\n"  # a distinct program (hash) of the same trace length
        progs.append(workload_trace(src, seed=30 + k))
    n = progs[0][0].shape[1]
    assert all(t.shape[1] == n for t, _ in progs)
    g = GpuProver(0, max_trace_len=n)
    try:
        for rep in range(2):
            for t, p in progs:
                proof, _, _, rc = g.prove(t, p, ProofOptions())
                assert rc == 0
                if rep == 1:
                    assert proof == oracle.prove(t, oracle_pub(oracle, p))[0]
        info = g.proof_info()
        assert info["hint_sets"] == 8 and info["hint_redos"] == 0, info
    finally:
        g.close()
