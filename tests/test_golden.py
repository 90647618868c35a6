"""Golden fixtures (tests/golden/, written by tools/gen_golden.py from the CPU oracle).

CPU: the fixtures' primitive vectors agree with Python big-int arithmetic (independent of the
oracle); the product VM (zk_vm_trace) regenerates every stored trace from the stored inputs;
the oracle regenerates every stored proof byte for byte and its verifier accepts them, and
rejects tampered copies.
GPU: the gfx950 prover reproduces every stored proof byte for byte through the C ABI.
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

from zkvm_amd import native
from zkvm_amd.prover import GpuProver, ProofOptions, make_pub_inputs, vm_trace
from zkvm_amd.workloads import ServerKey

GOLD = Path(__file__).resolve().parent / "golden"
DATA = json.loads((GOLD / "cases.json").read_text())
CASES = DATA["cases"]
PRIM = DATA["primitives"]
P = 2**128 - 45 * 2**40 + 1
IDS = [c["name"] for c in CASES]


def ints(hs):
    return [int(h, 16) for h in hs]


def blake3_spec(data: bytes) -> bytes:
    """Single-chunk BLAKE3-256 straight from the spec (inputs <= 1024 bytes), pure Python."""
    iv = [0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A, 0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19]
    perm = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]
    M = 0xFFFFFFFF

    def rotr(x, r):
        return ((x >> r) | (x << (32 - r))) & M

    def g(s, a, b, c, d, x, y):
        s[a] = (s[a] + s[b] + x) & M
        s[d] = rotr(s[d] ^ s[a], 16)
        s[c] = (s[c] + s[d]) & M
        s[b] = rotr(s[b] ^ s[c], 12)
        s[a] = (s[a] + s[b] + y) & M
        s[d] = rotr(s[d] ^ s[a], 8)
        s[c] = (s[c] + s[d]) & M
        s[b] = rotr(s[b] ^ s[c], 7)

    def compress(cv, block, blen, flags):
        m = [int.from_bytes(block[4 * i:4 * i + 4], "little") for i in range(16)]
        s = list(cv) + iv[:4] + [0, 0, blen, flags]
        for r in range(7):
            g(s, 0, 4, 8, 12, m[0], m[1]); g(s, 1, 5, 9, 13, m[2], m[3])
            g(s, 2, 6, 10, 14, m[4], m[5]); g(s, 3, 7, 11, 15, m[6], m[7])
            g(s, 0, 5, 10, 15, m[8], m[9]); g(s, 1, 6, 11, 12, m[10], m[11])
            g(s, 2, 7, 8, 13, m[12], m[13]); g(s, 3, 4, 9, 14, m[14], m[15])
            m = [m[p] for p in perm]
        return [s[i] ^ s[i + 8] for i in range(8)]

    assert len(data) <= 1024
    blocks = [data[i:i + 64] for i in range(0, len(data), 64)] or [b""]
    cv = iv
    for k, b in enumerate(blocks):
        flags = (1 if k == 0 else 0) | (2 | 8 if k == len(blocks) - 1 else 0)  # CHUNK_START, CHUNK_END|ROOT
        cv = compress(cv, b.ljust(64, b"\0"), len(b), flags)
    return b"".join(w.to_bytes(4, "little") for w in cv)


def test_primitive_vectors_against_bigint():
    a, b = ints(PRIM["a"]), ints(PRIM["b"])
    assert ints(PRIM["mul"]) == [x * y % P for x, y in zip(a, b)]
    assert ints(PRIM["add"]) == [(x + y) % P for x, y in zip(a, b)]
    assert ints(PRIM["sub"]) == [(x - y) % P for x, y in zip(a, b)]
    assert ints(PRIM["inv"]) == [pow(x, P - 2, P) for x in a if x]
    for k, r in PRIM["roots"].items():
        w = int(r, 16)
        k = int(k)
        assert pow(w, 2**k, P) == 1 and (k == 0 or pow(w, 2**(k - 1), P) != 1)
        assert w == pow(pow(3, (P - 1) >> 40, P), 2**(40 - k), P)
    for k, h in zip((1, 2, 4, 7, 8, 16, 21), PRIM["blake3_elems"]):
        data = b"".join(v.to_bytes(16, "little") for v in a[:k])
        assert blake3_spec(data).hex() == h
    coeffs, out = ints(PRIM["coset_lde_in"]), ints(PRIM["coset_lde_out"])
    w = pow(pow(3, (P - 1) >> 40, P), 2**(40 - 7), P)  # order-128 root
    for i in (0, 1, 5, 77, 127):
        x = 3 * pow(w, i, P) % P
        assert out[i] == sum(c * pow(x, j, P) for j, c in enumerate(coeffs)) % P


def test_primitive_vectors_against_oracle(oracle):
    a, b = ints(PRIM["a"]), ints(PRIM["b"])
    assert [oracle.fop("or_fmul", x, y) for x, y in zip(a, b)] == ints(PRIM["mul"])
    assert oracle.eval_coset(ints(PRIM["coset_lde_in"]), 128, 3) == ints(PRIM["coset_lde_out"])


def load_case(c):
    trace = np.load(GOLD / f"{c['name']}.trace.npy", allow_pickle=False)
    assert hashlib.sha256(trace.tobytes()).hexdigest() == c["trace_sha256"]
    proof = (GOLD / f"{c['name']}.proof").read_bytes()
    assert hashlib.sha256(proof).hexdigest() == c["proof_sha256"]
    pub = make_pub_inputs(ints(c["program_hash"]), ints(c["stack_outputs"]), c["lwe_size"], c["delta"])
    return trace, proof, pub


def options_of(c):
    o = c["options"]
    return ProofOptions(o["num_queries"], o["blowup"], o["grinding"], o["field_extension"], o["fri_folding"],
                        o["fri_rem_max_deg"])


def oracle_pub(oracle, c):
    return oracle.make_pub(ints(c["program_hash"]), ints(c["stack_outputs"]), c["lwe_size"], c["delta"])


@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_product_vm_regenerates_trace(c):
    trace, _, _ = load_case(c)
    sk = ServerKey(seed=0)  # only lwe_size / delta are read by the VM
    secret = [ints(ct) for ct in c["secret"]]
    got, outputs, h = vm_trace(c["source"], c["public"], secret, sk, ints(c["last_row"]))
    assert got.shape == trace.shape and np.array_equal(got, trace)
    assert outputs == ints(c["stack_outputs"]) and h == ints(c["program_hash"])


@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_oracle_regenerates_proof(oracle, c):
    trace, proof, _ = load_case(c)
    o = c["options"]
    opts = oracle.default_options(**o)
    got, rec, _ = oracle.prove(trace, oracle_pub(oracle, c), opts)
    assert bytes(rec.trace_root).hex() == c["trace_root"]
    assert bytes(rec.constraint_root).hex() == c["constraint_root"]
    assert bytes(rec.z).hex() == c["z"]
    assert [bytes(rec.fri_roots[i]).hex() for i in range(rec.num_fri_layers)] == c["fri_roots"]
    assert rec.pow_nonce == c["pow_nonce"]
    assert [rec.positions[i] for i in range(rec.num_positions)] == c["positions"]
    assert got == proof


@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_oracle_verifier_accepts_and_rejects(oracle, c):
    _, proof, _ = load_case(c)
    pub = oracle_pub(oracle, c)
    assert oracle.verify(proof, pub, 0) == (0, "")
    # tampering anywhere in the body must be caught (roots, queries, OOD frame, FRI, nonce)
    for off in (40, len(proof) // 3, len(proof) // 2, (2 * len(proof)) // 3, len(proof) - 12):
        bad = bytearray(proof)
        bad[off] ^= 0x01
        assert oracle.verify(bytes(bad), pub, 0)[0] != 0, f"tampered byte {off} accepted"
    # wrong public inputs
    wrong = oracle.make_pub(ints(c["program_hash"]), [1] + ints(c["stack_outputs"])[1:], c["lwe_size"], c["delta"])
    if ints(c["stack_outputs"])[0] != 1:
        assert oracle.verify(proof, wrong, 0)[0] != 0


@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_product_verifier_accepts_and_rejects(c):
    """zk_verify (the library's host verifier) on the golden proofs, tampered copies and wrong inputs."""
    from zkvm_amd.prover import verify
    _, proof, pub = load_case(c)
    assert verify(proof, pub, 0) == (0, "")
    for off in (40, len(proof) // 3, len(proof) // 2, (2 * len(proof)) // 3, len(proof) - 12):
        bad = bytearray(proof)
        bad[off] ^= 0x01
        rc, why = verify(bytes(bad), pub, 0)
        assert rc == native.ZK_ERR_VERIFY and why, f"tampered byte {off} accepted"
    assert verify(proof[:-1], pub, 0)[0] == native.ZK_ERR_VERIFY
    wrong = make_pub_inputs(ints(c["program_hash"]), [1] + ints(c["stack_outputs"])[1:], c["lwe_size"], c["delta"])
    if ints(c["stack_outputs"])[0] != 1:
        assert verify(proof, wrong, 0)[0] == native.ZK_ERR_VERIFY
    # conjectured security of the reference options is 95 bits
    if c["options"] == {"num_queries": 32, "blowup": 8, "grinding": 0, "field_extension": 1, "fri_folding": 8,
                        "fri_rem_max_deg": 127}:
        assert verify(proof, pub, 95)[0] == 0 and verify(proof, pub, 96)[0] == native.ZK_ERR_VERIFY


@pytest.mark.gpu
@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_gpu_reproduces_golden_proof(c):
    assert native.device_count() > 0
    trace, proof, pub = load_case(c)
    o = c["options"]
    g = GpuProver(0, max_trace_len=trace.shape[1], max_blowup=o["blowup"])
    try:
        got, rec, _, rc = g.prove(trace, pub, options_of(c), record=True)
    finally:
        g.close()
    assert rc == 0
    assert bytes(rec.trace_root).hex() == c["trace_root"]
    assert bytes(rec.constraint_root).hex() == c["constraint_root"]
    assert rec.pow_nonce == c["pow_nonce"]
    assert got == proof
