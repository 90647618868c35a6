"""GPU parity: the gfx950 path (libzkvm_gpu.so, via the C ABI) against the CPU oracle.

Bit-exact comparisons at sizes the oracle finishes in seconds (field ops, BLAKE3 rows, NTTs,
every stage intermediate, the full proof bytes), and at the benchmark size (n = 2^20) the
size-independent property that the GPU proof passes the oracle's verifier (Merkle openings,
out-of-domain AIR identity, DEEP, every FRI fold, remainder) with a composition-degree check.
"""
import ctypes as C
import random

import numpy as np
import pytest

from zkvm_amd import native
from zkvm_amd.prover import (GpuProver, ProofOptions, bytes_elems, elems_bytes, make_pub_inputs, vm_trace)
from zkvm_amd.workloads import LR_PROGRAM, cipher_mix_program, make_workload, push_add_program, ops_for_trace_len

pytestmark = pytest.mark.gpu
P = 2**128 - 45 * 2**40 + 1


@pytest.fixture(scope="module")
def gpu():
    assert native.device_count() > 0, "no GPU visible"
    g = GpuProver(0, max_trace_len=1 << 20, max_blowup=16)
    yield g
    g.close()


def test_runtime_is_the_one_the_library_links(gpu):
    """This GPU test process runs the library on the HIP runtime and RCCL it links (/opt/rocm), one copy of each:
    nothing in the suite imports torch, whose bundled ROCm 7.0 copies would otherwise serve it."""
    rt = native.runtime_info()
    print(rt)
    assert isinstance(rt["hip_runtime"], str) and rt["hip_runtime"].startswith("/opt/rocm"), rt
    assert isinstance(rt["rccl"], str) and rt["rccl"].startswith("/opt/rocm"), rt
    assert not rt["torch_loaded_first"] and len(native.mapped_files("libamdhip64.so")) == 1


def test_field_ops(gpu):
    rnd = random.Random(5)
    edge = [0, 1, 2, P - 1, P - 2, 2**64 - 1, 2**64, 2**127, P - 2**64, 45 * 2**40]
    a = edge + [rnd.randrange(P) for _ in range(4000)]
    b = list(reversed(edge)) + [rnd.randrange(P) for _ in range(4000)]
    for op, f in [(0, lambda x, y: (x + y) % P), (1, lambda x, y: (x - y) % P), (2, lambda x, y: x * y % P),
                  (3, lambda x, y: pow(x, P - 2, P) if x else 0)]:
        out = C.create_string_buffer(16 * len(a))
        native.check(native.lib().zk_diag_field_op(0, op, elems_bytes(a), elems_bytes(b), out, len(a)))
        got = bytes_elems(out.raw)
        assert all(g == f(x, y) for g, x, y in zip(got, a, b)), f"op {op}"
    e = [rnd.randrange(2**128) for _ in a]
    out = C.create_string_buffer(16 * len(a))
    native.check(native.lib().zk_diag_field_op(0, 4, elems_bytes(a), elems_bytes(e), out, len(a)))
    assert bytes_elems(out.raw) == [pow(x, y, P) for x, y in zip(a, e)]


def test_lazy_field_forms(gpu):
    """The NTT's partially reduced forms (f128.hpp fe_add_lazy / fe_sub / fe_canon and the multiplies): the
    first operand may be any value below 2^128, the second is canonical; results stay below 2^128 and are
    congruent mod p.  Non-canonical values are rare on random data (~2^-82 per sum), so the edges are crafted."""
    rnd = random.Random(11)
    hi = [2**128 - 1, 2**128 - 2, P, P + 1, 2**128 - 45 * 2**40, P - 1, 2**127, 0]
    a = [x for x in hi for _ in hi] + [rnd.randrange(P, 2**128) for _ in range(2000)] + [rnd.randrange(2**128) for _ in range(2000)]
    bl = [P - 1, P - 2, 0, 1, 2**127, P - 2**64, 45 * 2**40, 2**64 - 1]
    b = [y for _ in hi for y in bl] + [rnd.choice([P - 1, rnd.randrange(P)]) for _ in range(4000)]

    def run(op, xs, ys):
        out = C.create_string_buffer(16 * len(xs))
        native.check(native.lib().zk_diag_field_op(0, op, elems_bytes(xs), elems_bytes(ys), out, len(xs)))
        return bytes_elems(out.raw)

    for op, f in [(5, lambda x, y: x + y), (1, lambda x, y: x - y), (2, lambda x, y: x * y), (7, lambda x, y: x * y)]:
        for g, x, y in zip(run(op, a, b), a, b):
            assert 0 <= g < 2**128 and g % P == f(x, y) % P, (op, x, y, g)
            if op in (2, 7):
                assert g < P, (op, x, y, g)  # multiplies return canonical values
    assert run(6, a, b) == [x % P for x in a]


def test_butterfly_addsub2_forms(gpu):
    """The NTT butterflies' two sums and two differences in one interleaved asm block (f128.hpp addsub2_v,
    addsub_asm.hpp from tools/gen_addsub_asm.py), all three forms, bit for bit against Python integers: a + b
    canonical, or lazy (any first operand < 2^128: a + b, minus 2^128 - C on overflow), and a - b (+ p on a borrow).
    Lane t returns output t % 4 of (x + y, x - y, x2 + y2, x2 - y2), x2 / y2 the inputs of the mirrored lane."""
    rnd = random.Random(12)
    C128 = 2**128 - P
    canon = [0, 1, P - 1, P - 2, 2**64 - 1, 2**64, 2**127, P - 2**64, 45 * 2**40, 2**128 - 2**96 - 1]
    anyv = canon + [2**128 - 1, 2**128 - 2, P, P + 1, 2**128 - 45 * 2**40]

    def lazy(x, y):
        s = x + y
        return s if s < 2**128 else s - 2**128 + C128

    def sub(x, y):
        return x - y if x >= y else x - y + P

    for op, lz1, lz2 in ((8, False, False), (9, True, True), (10, True, False)):
        pool1, pool2 = (anyv if lz1 else canon), (anyv if lz2 else canon)
        m = 4096
        a = [pool1[i % len(pool1)] if i < 400 else rnd.choice([rnd.randrange(P), rnd.choice(pool1)]) for i in range(m)]
        b = [canon[(i // len(pool1)) % len(canon)] if i < 400 else rnd.choice([rnd.randrange(P), P - 1]) for i in range(m)]
        # the mirrored lanes feed the second pair: lanes whose mirror would hand a lazy value to a canonical-only slot
        # take canonical first operands
        if not lz2:
            a[m // 2:] = [x % P for x in a[m // 2:]]
            if not lz1:
                a = [x % P for x in a]
        out = C.create_string_buffer(16 * m)
        native.check(native.lib().zk_diag_field_op(0, op, elems_bytes(a), elems_bytes(b), out, m))
        got = bytes_elems(out.raw)
        for t in range(m):
            x, y, x2, y2 = a[t], b[t], a[m - 1 - t], b[m - 1 - t]
            if (not lz1 and x >= P) or (not lz2 and x2 >= P):
                continue  # outside that form's contract
            want = [lazy(x, y) if lz1 else (x + y) % P, sub(x, y), lazy(x2, y2) if lz2 else (x2 + y2) % P, sub(x2, y2)]
            assert got[t] == want[t & 3], (op, t, x, y, x2, y2, got[t], want[t & 3])


@pytest.mark.parametrize("k", [1, 4, 7, 8, 28])
def test_blake3_rows(gpu, oracle, k):
    rnd = random.Random(k)
    rows = [[rnd.randrange(P) for _ in range(k)] for _ in range(300)]
    out = C.create_string_buffer(32 * len(rows))
    native.check(native.lib().zk_diag_blake3_rows(0, elems_bytes([v for r in rows for v in r]), k, len(rows), out))
    for i, r in enumerate(rows):
        assert out.raw[32 * i:32 * i + 32] == oracle.blake3(elems_bytes(r))


@pytest.mark.parametrize("log_n", [2, 4, 7, 10, 12, 13, 14, 16])
def test_ntt(gpu, oracle, log_n):
    n = 1 << log_n
    rnd = random.Random(log_n)
    batch = 3
    vals = [rnd.randrange(P) for _ in range(n * batch)]
    out = C.create_string_buffer(16 * n * batch)
    # forward over the coset 3 * <w_n>
    native.check(native.lib().zk_diag_ntt(0, elems_bytes(vals), n, batch, 0, elems_bytes([3]), out))
    got = bytes_elems(out.raw)
    for b in range(batch):
        assert got[b * n:(b + 1) * n] == oracle.eval_coset(vals[b * n:(b + 1) * n], n, 3), f"forward batch {b}"
    # inverse over <w_n>
    native.check(native.lib().zk_diag_ntt(0, elems_bytes(vals), n, batch, 1, None, out))
    got = bytes_elems(out.raw)
    for b in range(batch):
        assert got[b * n:(b + 1) * n] == oracle.interp_coset(vals[b * n:(b + 1) * n], 1), f"inverse batch {b}"


def _random_elems_bytes(count, seed):
    """count canonical field elements as 16-byte LE words (hi < 2^64 - 1 keeps every value below p)."""
    rng = np.random.default_rng(seed)
    a = np.empty((count, 2), dtype=np.uint64)
    a[:, 0] = rng.integers(0, 2**64, size=count, dtype=np.uint64)
    a[:, 1] = rng.integers(0, 2**64 - 1, size=count, dtype=np.uint64)
    return a.tobytes()


@pytest.mark.parametrize("log_n", [20, 21, 22])
def test_ntt_four_step_splits(oracle, log_n):
    """Sizes whose four-step split is uneven or LOGM-odd (ntt_log_n2: 2^21 -> 11/10, 2^22 -> 12/10),
    one column, against the oracle's radix-2 transforms (bytes compared directly)."""
    n = 1 << log_n
    vals = _random_elems_bytes(n, log_n)
    out = C.create_string_buffer(16 * n)
    native.check(native.lib().zk_diag_ntt(0, vals, n, 1, 0, elems_bytes([3]), out))
    ref = C.create_string_buffer(16 * n)
    assert oracle.lib().or_eval_coset(vals, n, n, elems_bytes([3]), ref) == 0
    assert out.raw == ref.raw, "forward coset NTT differs"
    native.check(native.lib().zk_diag_ntt(0, vals, n, 1, 1, None, out))
    buf = C.create_string_buffer(vals, 16 * n)
    assert oracle.lib().or_interp_coset(buf, n, elems_bytes([1])) == 0
    assert out.raw == buf.raw, "inverse NTT differs"


@pytest.mark.parametrize("log_n", [20, 21, 22])
def test_ntt_lazy_edge_values(oracle, log_n):
    """Columns drawn from {0, 1, 2, p - 2, p - 1}: pass-1 butterfly sums such as (p - 1) + 2 = p + 1 stay
    partially reduced in the tile (ZK_NTT_LAZY), and the wave-uniform j = 0 rounds, which skip their unit
    twiddle multiplies, must still hand canonical second operands to the lazy add / subtract (a
    later j = 0 wave computed 0 - (p + 1) wrongly).  Random canonical data almost never reaches those values,
    so the inverse (trace interpolation) and the forward coset transform are checked on such columns."""
    n = 1 << log_n
    rng = np.random.default_rng(100 + log_n)
    pick = np.array([[0, 0], [1, 0], [2, 0], [(P - 2) % 2**64, (P - 2) >> 64], [(P - 1) % 2**64, (P - 1) >> 64]],
                    dtype=np.uint64)
    vals = pick[rng.integers(0, 5, size=n)].tobytes()
    out = C.create_string_buffer(16 * n)
    native.check(native.lib().zk_diag_ntt(0, vals, n, 1, 1, None, out))
    buf = C.create_string_buffer(vals, 16 * n)
    assert oracle.lib().or_interp_coset(buf, n, elems_bytes([1])) == 0
    assert out.raw == buf.raw, "inverse NTT differs on edge-valued input"
    native.check(native.lib().zk_diag_ntt(0, vals, n, 1, 0, elems_bytes([3]), out))
    ref = C.create_string_buffer(16 * n)
    assert oracle.lib().or_eval_coset(vals, n, n, elems_bytes([3]), ref) == 0
    assert out.raw == ref.raw, "forward coset NTT differs on edge-valued input"


def workload_trace(source, seed=3):
    w = make_workload(source, seed=seed)
    trace, outputs, h = vm_trace(source, w.public, w.secret, w.server_key, w.last_row)
    return trace, make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)


def oracle_pub(oracle, pub):
    p = oracle.PubInputs()
    C.memmove(p.program_hash, bytes(pub.program_hash), 32)
    C.memmove(p.stack_outputs, bytes(pub.stack_outputs), 256)
    p.lwe_size, p.delta = pub.lwe_size, pub.delta
    return p


def compare_records(rec, orec):
    for name, _ in type(orec)._fields_:
        assert bytes(getattr(rec, name)) == bytes(getattr(orec, name)) if not isinstance(getattr(orec, name), int) \
            else getattr(rec, name) == getattr(orec, name), f"record field {name} differs"


CASES = [("push.5\npush.3\nadd", ProofOptions()), (LR_PROGRAM, ProofOptions()),
         (push_add_program(200), ProofOptions()), (cipher_mix_program(60)[0], ProofOptions()),
         (cipher_mix_program(60)[0], ProofOptions(num_queries=40, blowup_factor=16, fri_folding_factor=4,
                                                  fri_remainder_max_degree=31, grinding_factor=4)),
         (ops_for_trace_len(14, "cipher"), ProofOptions()),
         # four-step coset-table LDE with 16 cosets: two 8-coset launches per pass
         (ops_for_trace_len(13, "cipher"), ProofOptions(num_queries=28, blowup_factor=16)),
         (LR_PROGRAM, ProofOptions(num_queries=20, grinding_factor=18)),  # GPU proof-of-work search
         # option maxima: 255 queries (many shared Merkle paths in the batch openings), remainder degree 255
         (cipher_mix_program(60)[0], ProofOptions(num_queries=255, fri_remainder_max_degree=255)),
         (cipher_mix_program(60)[0], ProofOptions(num_queries=255, fri_folding_factor=2, fri_remainder_max_degree=7))]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_full_proof_matches_oracle(gpu, oracle, case):
    source, options = CASES[case]
    trace, pub = workload_trace(source, seed=case)
    proof, rec, _, rc = gpu.prove(trace, pub, options, record=True)
    assert rc == 0
    oopt = oracle.default_options(num_queries=options.num_queries, blowup=options.blowup_factor,
                                  grinding=options.grinding_factor, fri_folding=options.fri_folding_factor,
                                  fri_rem_max_deg=options.fri_remainder_max_degree)
    opub = oracle_pub(oracle, pub)
    oproof, orec, _ = oracle.prove(trace, opub, oopt)
    compare_records(rec, orec)
    assert proof == oproof
    assert oracle.verify(proof, opub, 0) == (0, "")


def test_config1_pushadd_2_16_bit_exact(gpu, oracle):
    """BASELINE.json configs[1]: a 2^16-step Push/Add program, full prove on one GPU, proof bytes
    identical to the CPU prover (the oracle, ~10 s)."""
    src = ops_for_trace_len(16, "pushadd")
    trace, pub = workload_trace(src, seed=16)
    assert trace.shape[1] == 1 << 16
    proof, rec, _, rc = gpu.prove(trace, pub, ProofOptions(), record=True)
    assert rc == 0
    opub = oracle_pub(oracle, pub)
    oproof, orec, _ = oracle.prove(trace, opub)
    compare_records(rec, orec)
    assert proof == oproof
    assert oracle.verify(proof, opub, 95) == (0, "")


def test_stage_dumps_match_oracle(gpu, oracle):
    trace, pub = workload_trace(cipher_mix_program(30)[0], seed=11)
    names = ("trace_polys", "trace_lde", "trace_leaves", "composition", "comp_polys", "comp_lde", "deep", "fri_layer1")
    _, _, dumps, _ = gpu.prove(trace, pub, ProofOptions(), dump=names)
    _, orec, odumps = oracle.prove(trace, oracle_pub(oracle, pub), want=names)
    n = trace.shape[1]
    C_ = orec.num_ccols
    trim = {"comp_polys": C_ * n, "comp_lde": 8 * n * C_}
    for name in names:
        k = trim.get(name, len(odumps[name]))
        if name == "comp_lde":
            assert np.array_equal(dumps[name][:k], odumps[name][:k]), name
        else:
            assert np.array_equal(dumps[name][:k], odumps[name][:k]), name


def test_quadratic_stage_dumps_match_oracle(gpu, oracle):
    """FieldExtension::Quadratic: every stage (a components of the E-valued ones, both planes of the
    composition columns) equals the oracle's."""
    trace, pub = workload_trace(cipher_mix_program(30)[0], seed=12)
    names = ("composition", "comp_polys", "comp_lde", "deep", "fri_layer1")
    opts = ProofOptions(32, 8, 0, 2, 8, 127)
    proof, _, dumps, rc = gpu.prove(trace, pub, opts, dump=names)
    assert rc == 0
    oproof, orec, odumps = oracle.prove(trace, oracle_pub(oracle, pub), oracle.default_options(field_extension=2),
                                        want=names)
    n = trace.shape[1]
    ck = 2 * orec.num_ccols
    trim = {"comp_polys": ck * n, "comp_lde": 8 * n * ck}
    for name in names:
        k = trim.get(name, len(odumps[name]))
        assert np.array_equal(dumps[name][:k], odumps[name][:k]), name
    assert proof == oproof


def test_config5_quadratic_128_bit(gpu, oracle):
    """SURVEY config 5 at 2^14: FieldExtension::Quadratic with 43 queries reaches 128-bit conjectured
    security; proof bytes identical to the oracle's and accepted by both verifiers at 128 bits."""
    from zkvm_amd.prover import verify
    src = ops_for_trace_len(14, "pushadd")
    trace, pub = workload_trace(src, seed=14)
    opts = ProofOptions(43, 8, 0, 2, 8, 127)
    proof, rec, _, rc = gpu.prove(trace, pub, opts, record=True)
    assert rc == 0
    opub = oracle_pub(oracle, pub)
    oproof, orec, _ = oracle.prove(trace, opub, oracle.default_options(num_queries=43, field_extension=2))
    compare_records(rec, orec)
    assert proof == oproof
    assert oracle.verify(proof, opub, 128) == (0, "")
    assert verify(proof, pub, 128) == (0, "")
    assert verify(proof, pub, 129)[0] == native.ZK_ERR_VERIFY


def test_plug_points(gpu, oracle):
    """zk_lde_new / read_frame / query / eval_constraints against the oracle's stages."""
    trace, pub = workload_trace(LR_PROGRAM, seed=2)
    n = trace.shape[1]
    L = native.lib()
    h = C.c_void_p()
    root = C.create_string_buffer(32)
    tb = np.ascontiguousarray(trace)
    native.check(L.zk_lde_new(gpu.handle, tb.ctypes.data, 28, n, 8, C.byref(h), root))
    _, orec, od = oracle.prove(trace, oracle_pub(oracle, pub), want=("trace_lde", "composition"))
    assert root.raw == bytes(orec.trace_root)
    lde = od["trace_lde"].reshape(8 * n, 28, 2)
    cur, nxt = C.create_string_buffer(28 * 16), C.create_string_buffer(28 * 16)
    for step in (0, 5, 8 * n - 3):
        native.check(L.zk_lde_read_frame(h, step, cur, nxt))
        assert cur.raw == lde[step].tobytes() and nxt.raw == lde[(step + 8) % (8 * n)].tobytes()
    pos = (C.c_uint64 * 3)(1, 17, 900)
    rows = C.create_string_buffer(3 * 28 * 16)
    plen = C.c_size_t(1 << 16)
    pbuf = C.create_string_buffer(1 << 16)
    native.check(L.zk_lde_query(h, pos, 3, rows, pbuf, C.byref(plen)))
    assert rows.raw == b"".join(lde[p].tobytes() for p in (1, 17, 900))
    out = C.create_string_buffer(16 * 8 * n)
    native.check(L.zk_eval_constraints(h, C.byref(pub), bytes(orec.coeff_t), bytes(orec.coeff_b), out))
    assert out.raw == od["composition"].tobytes()
    L.zk_lde_free(h)


def test_plug_point_constraint_commitment(gpu, oracle):
    """zk_commit_composition / zk_comp_query (build_constraint_commitment) against the oracle's composition
    column polynomials, composition LDE and constraint root."""
    trace, pub = workload_trace(cipher_mix_program(60)[0], seed=7)
    n = trace.shape[1]
    L = native.lib()
    h = C.c_void_p()
    tb = np.ascontiguousarray(trace)
    native.check(L.zk_lde_new(gpu.handle, tb.ctypes.data, 28, n, 8, C.byref(h), C.create_string_buffer(32)))
    _, orec, od = oracle.prove(trace, oracle_pub(oracle, pub), want=("composition", "comp_polys", "comp_lde"))
    ncols = orec.num_ccols
    comp = np.ascontiguousarray(od["composition"])
    cc, root = C.c_void_p(), C.create_string_buffer(32)
    polys = C.create_string_buffer(16 * ncols * n)
    native.check(L.zk_commit_composition(h, comp.ctypes.data, ncols, C.byref(cc), root, polys))
    assert root.raw == bytes(orec.constraint_root)
    assert polys.raw == od["comp_polys"].reshape(-1, 2)[: ncols * n].tobytes()
    clde = od["comp_lde"].reshape(-1, 2)[: 8 * n * ncols].reshape(8 * n, ncols, 2)
    pos = (C.c_uint64 * 4)(0, 3, 8 * n - 1, 77)
    rows = C.create_string_buffer(4 * ncols * 16)
    plen = C.c_size_t(1 << 16)
    pbuf = C.create_string_buffer(1 << 16)
    native.check(L.zk_comp_query(cc, pos, 4, rows, pbuf, C.byref(plen)))
    assert rows.raw == b"".join(clde[p].tobytes() for p in (0, 3, 8 * n - 1, 77))
    assert 0 < plen.value < (1 << 16)
    L.zk_comp_free(cc)
    # a composition of too high a degree is refused: more columns' worth of coefficients than num_cols
    rc = L.zk_commit_composition(h, comp.ctypes.data, ncols - 1, C.byref(cc), root, None)
    assert rc == native.ZK_ERR_DEGREE
    L.zk_lde_free(h)


def test_invalid_trace_is_reported(gpu):
    trace, pub = workload_trace(LR_PROGRAM, seed=4)
    bad = trace.copy()
    bad[12, 10, 0] ^= 1  # break a stack transition mid-program
    _, _, _, rc = gpu.prove(bad, pub, ProofOptions(), allow_degree_error=True)
    assert rc == native.ZK_ERR_DEGREE


@pytest.mark.parametrize("ext", [1, 2])
def test_failed_assertion_is_reported(gpu, ext):
    """Public stack outputs that the trace does not end with: a step-(n-2) assertion fails.  The prover adds
    the assertion terms in coefficient form; the division remainder must raise the degree error."""
    trace, pub = workload_trace(LR_PROGRAM, seed=5)
    wrong = native.PubInputs()
    C.memmove(C.byref(wrong), C.byref(pub), C.sizeof(pub))
    wrong.stack_outputs[0] ^= 1
    _, _, _, rc = gpu.prove(trace, wrong, ProofOptions(field_extension=ext), allow_degree_error=True)
    assert rc == native.ZK_ERR_DEGREE
    # and the unmodified public inputs prove
    _, _, _, rc = gpu.prove(trace, pub, ProofOptions(field_extension=ext))
    assert rc == 0


def test_bench_size_proof_verifies(gpu, oracle):
    """configs[2] size: 2^20-step ciphertext program; the GPU proof must verify (size-independent check)."""
    source = ops_for_trace_len(20, "cipher")
    trace, pub = workload_trace(source, seed=20)
    assert trace.shape[1] == 1 << 20
    proof, rec, _, rc = gpu.prove(trace, pub, ProofOptions(), record=True)
    assert rc == 0
    assert rec.num_fri_layers == 5 and rec.remainder_len == 32
    assert oracle.verify(proof, oracle_pub(oracle, pub), 95) == (0, "")
    # proof is deterministic for a fixed trace
    proof2, _, _, _ = gpu.prove(trace, pub, ProofOptions())
    assert proof2 == proof


def test_2_22_proof_verifies(oracle):
    """configs[3] size on one GPU: a 2^22-step cipher-mix proof (the four-step NTTs take the 12/10 split
    here) verifies with zk_verify and the oracle's verifier."""
    from zkvm_amd.prover import verify
    source = ops_for_trace_len(22, "cipher")
    trace, pub = workload_trace(source, seed=22)
    assert trace.shape[1] == 1 << 22
    g = GpuProver(0, max_trace_len=1 << 22)
    try:
        proof, _, _, rc = g.prove(trace, pub, ProofOptions())
    finally:
        g.close()
    assert rc == 0
    assert verify(proof, pub, 95) == (0, "")
    assert oracle.verify(proof, oracle_pub(oracle, pub), 95) == (0, "")


def test_reference_vm_prove_and_verify(gpu):
    """vm/src/lib.rs:47-99 (test_prove) through the GPU prover: the same program, inputs and LWE
    parameters; the decrypted output is (a + x) * 3 and the proof verifies at 95 bits (zk_verify, and
    the oracle's verifier)."""
    from zkvm_amd.prover import prove, verify
    from zkvm_amd.workloads import LweParameters, ServerKey, rand_field
    import numpy as np
    src = "read2\nread\nsadd\npush.1\npush.2\nadd\nsmul\n"
    a, b, clear_x = 1, 3, 2
    sk = ServerKey(LweParameters(8, 128, 4, 2.412_390_240_121_573e-5), seed=99)
    x = sk.encrypt(clear_x)
    last_row = [rand_field(np.random.default_rng(5), lo=1) for _ in range(28)]
    h, output, proof = prove(src, [a, b], [x], sk, last_row, gpu=gpu)
    assert sk.decrypt(output[:5]) == (a + clear_x) * 3
    pub = make_pub_inputs(h, output, sk.lwe_size(), sk.parameters.delta)
    assert verify(proof, pub, 95) == (0, "")


@pytest.mark.parametrize("k", [1, 2, 3])
def test_other_lwe_sizes(gpu, oracle, k):
    """Ciphertexts of k + 1 elements (lwe_size 2..4 instead of the example's 5).  The reference AIR hard-codes
    the 5-element ciphertext in its depth and read2 constraints (tests/test_oracle_vm_air.py), so such traces
    are refused -- here and by the oracle, both with a degree error -- but the evaluator's lwe_size loop must
    still agree with the oracle: the zk_eval_constraints plug point reproduces the oracle's composition
    values (every CE step) at lwe_size = k + 1."""
    from zkvm_amd.workloads import LweParameters
    src = cipher_mix_program(12)[0]
    w = make_workload(src, seed=30 + k, params=LweParameters(8, 128, k, 2.412_390_240_121_573e-5))
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    assert pub.lwe_size == k + 1
    _, _, _, rc = gpu.prove(trace, pub, ProofOptions(), allow_degree_error=True)
    assert rc == native.ZK_ERR_DEGREE
    orc, _, orec, od = oracle.prove_rc(trace, oracle_pub(oracle, pub), want=("composition",))
    assert orc == native.ZK_ERR_DEGREE
    n = trace.shape[1]
    L = native.lib()
    hnd = C.c_void_p()
    tb = np.ascontiguousarray(trace)
    native.check(L.zk_lde_new(gpu.handle, tb.ctypes.data, 28, n, 8, C.byref(hnd), C.create_string_buffer(32)))
    try:
        out = C.create_string_buffer(16 * 8 * n)
        native.check(L.zk_eval_constraints(hnd, C.byref(pub), bytes(orec.coeff_t), bytes(orec.coeff_b), out))
        assert out.raw == od["composition"].tobytes()
    finally:
        L.zk_lde_free(hnd)


@pytest.mark.parametrize("grinding", [33, 64, 255])
def test_grinding_factor_bound(gpu, grinding):
    """winter-air ProofOptions caps grinding_factor at 32: larger values are refused up front (a search for
    more than 64 trailing zero bits would never end; the proof stores the factor in one byte)."""
    trace, pub = workload_trace(LR_PROGRAM, seed=4)
    with pytest.raises(native.ZkError) as e:
        gpu.prove(trace, pub, ProofOptions(grinding_factor=grinding))
    assert e.value.code == native.ZK_ERR_INVALID_ARG and "grinding" in str(e.value)


@pytest.mark.parametrize("field,value", [("field_extension", 3), ("blowup_factor", 4), ("blowup_factor", 12),
                                         ("fri_folding_factor", 3), ("fri_remainder_max_degree", 100),
                                         ("num_queries", 0)])
def test_unsupported_options_refused(gpu, field, value):
    """Options winterfell 0.9 would not accept (or this prover does not implement) are refused with
    ZK_ERR_INVALID_ARG before any device work."""
    trace, pub = workload_trace(LR_PROGRAM, seed=4)
    with pytest.raises(native.ZkError) as e:
        gpu.prove(trace, pub, ProofOptions(**{field: value}))
    assert e.value.code == native.ZK_ERR_INVALID_ARG


def test_proof_buffer_too_small_then_proof(gpu, oracle):
    """A proof buffer too small for the proof gives ZK_ERR_BUFFER_TOO_SMALL (nothing written past it); the next
    proof with room is the oracle's."""
    trace, pub = workload_trace(LR_PROGRAM, seed=5)
    gpu._proof_buf = C.create_string_buffer(64)
    try:
        with pytest.raises(native.ZkError) as e:
            gpu.prove(trace, pub, ProofOptions())
        assert e.value.code == native.ZK_ERR_BUFFER_TOO_SMALL
    finally:
        gpu._proof_buf = None
    proof, _, _, rc = gpu.prove(trace, pub, ProofOptions())
    assert rc == 0 and proof == oracle.prove(trace, oracle_pub(oracle, pub))[0]


def test_error_then_proof_is_unchanged(gpu, oracle):
    """A proof that fails part-way (degree error after staged reads) leaves nothing pending in the
    prover's pinned staging area: the next proof is byte-identical to the oracle's."""
    trace, pub = workload_trace(LR_PROGRAM, seed=6)
    bad = trace.copy()
    bad[12, 10, 0] ^= 1
    _, _, _, rc = gpu.prove(bad, pub, ProofOptions(), allow_degree_error=True)
    assert rc == native.ZK_ERR_DEGREE
    proof, _, _, rc = gpu.prove(trace, pub, ProofOptions())
    assert rc == 0
    oproof, _, _ = oracle.prove(trace, oracle_pub(oracle, pub))
    assert proof == oproof


def test_provers_on_every_device_agree(oracle):
    """__constant__ tables (Rescue MDS / inverse MDS) are per device: a prover on each visible GPU of one
    process, created after another device already proved, gives the same proof bytes."""
    n_dev = native.device_count()
    trace, pub = workload_trace(LR_PROGRAM, seed=8)
    oproof, _, _ = oracle.prove(trace, oracle_pub(oracle, pub))
    for dev in range(min(n_dev, 8)):
        g = GpuProver(dev, max_trace_len=trace.shape[1])
        try:
            proof, _, _, rc = g.prove(trace, pub, ProofOptions())
        finally:
            g.close()
        assert rc == 0 and proof == oproof, f"device {dev}"


# ---------------------------------------------------------------- full-size pins (BASELINE configs[2], [3], [4])
from golden_large import LARGE_CASES, check_large_proof, large_inputs  # noqa: E402


@pytest.mark.parametrize("name", [c["name"] for c in LARGE_CASES])
def test_full_size_proof_matches_oracle_pin(oracle, name):
    """configs[2] (2^20, reference options), configs[4] (2^20, 43 queries over the quadratic extension, 128 bits)
    and configs[3]'s 2^22 trace on one GPU: the proof from the host-resident trace is byte-identical to the
    oracle's (sha256, roots, query positions) and both verifiers accept it at the config's security."""
    c = next(c for c in LARGE_CASES if c["name"] == name)
    ht, trace, pub, opts = large_inputs(c)
    g = GpuProver(0, max_trace_len=1 << c["log_n"])
    try:
        proof, rec, _, rc = g.prove(trace, pub, opts, record=True)
    finally:
        g.close()
        ht.close()
    assert rc == 0
    check_large_proof(c, proof, rec, pub, oracle)


def test_largest_single_gpu_trace_2p23(oracle):
    """The largest trace this build proves on one GPU: 2^23 steps (a ~100 GB full prover of the 288 GB HBM; every
    LDE-domain index of 28 x 2^26 elements still fits the kernels' 32-bit grid arithmetic).  No oracle pin at this
    size (the CPU oracle would need ~30 GB and ~15 min): the proof from the page-locked host trace must verify with
    both verifiers, and its trace root must not depend on the upload path (device-resident proof: same bytes)."""
    from golden_large import oracle_pub
    from zkvm_amd.prover import HostTrace, Program, verify
    src = ops_for_trace_len(23, "cipher")
    w = make_workload(src, seed=2300)
    prog = Program(src)
    ht = HostTrace(prog.trace_len)
    g = None
    try:
        trace, outputs = prog.trace(w.public, w.secret, w.server_key, w.last_row, out=ht)
        assert trace.shape[1] == 1 << 23
        pub = make_pub_inputs(prog.hash, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
        g = GpuProver(0, max_trace_len=1 << 23)
        proof, _, _, rc = g.prove(trace, pub, ProofOptions())
        assert rc == 0
        d, _ = g.upload_trace(trace)
        proof_dev, _, _, rc2 = g.prove_device(d, 1 << 23, pub, ProofOptions())
        assert rc2 == 0 and proof_dev == proof
    finally:
        if g is not None:
            g.close()
        prog.close()
        ht.close()
    assert verify(proof, pub, 95) == (0, "")
    assert oracle.verify(proof, oracle_pub(oracle, pub), 95) == (0, "")


def test_host_trace_memory_outlives_its_owner(gpu, oracle):
    """A trace written into a HostTrace that is dropped at once (`trace, o = prog.trace(..., out=HostTrace(n))`)
    keeps its page-locked block alive: the array's base chain owns the allocation, so proving from it reads live
    memory and gives the oracle's proof."""
    import gc

    from golden_large import oracle_pub
    from zkvm_amd.prover import HostTrace, Program, _PinnedBlock
    w = make_workload(LR_PROGRAM, seed=21)
    prog = Program(LR_PROGRAM)
    trace, outputs = prog.trace(w.public, w.secret, w.server_key, w.last_row, out=HostTrace(prog.trace_len))
    h = prog.hash
    prog.close()
    gc.collect()
    base = trace
    while base is not None and not isinstance(base, _PinnedBlock):
        base = getattr(base, "base", None)
    assert isinstance(base, _PinnedBlock) and base.ptr
    scratch = [np.full((28, trace.shape[1], 2), 0xAB, dtype=np.uint64) for _ in range(8)]  # reuse freed pages, if any
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    proof, _, _, rc = gpu.prove(trace, pub, ProofOptions())
    del scratch
    assert rc == 0
    ref, _, _ = oracle.prove(np.array(trace), oracle_pub(oracle, pub))
    assert proof == ref


@pytest.mark.parametrize("path", ["host", "device"])
def test_sparse_column_detection(gpu, oracle, path):
    """Sparse trace columns (zero in every row but the last: SparseCols) skip their NTTs.  A 2^14 trace with the
    VM's sparse registers (s11..s15), one of them with a zero last row too, one made dense by a single middle entry,
    and s10 zeroed but for its last row (sparse) -- edits in columns no constraint or assertion reads, so the trace
    still satisfies the AIR: the proof equals the oracle's, from the host trace (upload groups) and from HBM."""
    trace, pub = workload_trace(ops_for_trace_len(14, "cipher"), seed=14)
    n = trace.shape[1]
    t = trace.copy()
    assert not t[23:28, : n - 1].any()  # the cipher mix never reaches stack depth 12
    t[25, n - 1] = 0                     # sparse with a zero last row
    t[27, 5] = [7, 0]                    # one entry in the middle: dense
    t[22, : n - 1] = 0                   # s10, zeroed but for its last row: sparse
    oproof, orec, _ = oracle.prove(t, oracle_pub(oracle, pub))
    if path == "host":
        proof, rec, _, rc = gpu.prove(t, pub, ProofOptions(), record=True)
    else:
        d, _ = gpu.upload_trace(t)
        proof, rec, _, rc = gpu.prove_device(d, n, pub, ProofOptions(), record=True)
    assert rc == 0
    assert bytes(rec.trace_root) == bytes(orec.trace_root)
    assert proof == oproof


@pytest.mark.parametrize("schedule", ["auto", "throughput", "latency"])
def test_narrow_columns_learned_and_refuted(oracle, schedule):
    """Narrow columns (a host-resident trace's columns that the previous proof of the same length found to hold 8- or
    32-bit values before the last row go up packed, each value checked on the host; one that does not fit goes up
    whole): the proofs of a trace, of the same trace again (packed), and of edits that break the 8-bit and then the
    32-bit class of a learned column -- each equal to the oracle's, with the upload shrinking once the hint is
    learned.  On each upload schedule (zk_prover_set_upload_schedule: auto -- latency, this prover being alone --,
    throughput: two packed parts through the copy engine; latency: parts of 1, 2, 2, .. columns expanded from pinned
    memory)."""
    trace, pub = workload_trace(ops_for_trace_len(14, "cipher"), seed=16)
    n = trace.shape[1]
    small = trace.copy()
    small[27, : n - 1] = 0
    small[27, 5:200, 0] = np.arange(5, 200) % 251 + 1  # s15 (read by no constraint): 8-bit values
    wide8 = small.copy()
    wide8[27, 77] = [300, 0]                            # no longer 8-bit
    wide32 = small.copy()
    wide32[27, 78] = [1 << 40, 0]                       # no longer 32-bit
    g = GpuProver(0, max_trace_len=n)
    g.set_upload_schedule(schedule)
    try:
        stats = []
        for t in (trace, trace, small, small, wide8, wide8, wide32, small):
            proof, _, _, rc = g.prove(t, pub, ProofOptions())
            assert rc == 0
            oproof, _, _ = oracle.prove(t, oracle_pub(oracle, pub))
            assert proof == oproof
            stats.append(g.upload_stats())
    finally:
        g.close()
    full = 28 * n * 16
    assert stats[0]["bytes"] == full and not stats[0]["narrow8"]
    # learned: the bit columns go up as bytes, the clock (learned as 32-bit) is derived from the AIR, 5 sparse columns
    # not at all
    assert set(range(1, 7)) <= set(stats[1]["narrow8"]) and stats[1]["derived"] == [0]
    # nothing of the sparse or derived columns goes up (their last row aside), the narrow ones as 1 or 4 bytes per row
    st = stats[1]
    wide = 28 - len(st["sparse"]) - len(st["narrow8"]) - len(st["narrow32"]) - len(st["derived"])
    assert len(st["sparse"]) >= 5
    assert st["bytes"] == wide * n * 16 + (len(st["narrow8"]) + 4 * len(st["narrow32"])) * n
    assert 27 in stats[3]["narrow8"]                   # small: s15 learned as 8-bit
    assert 27 not in stats[4]["narrow8"] + stats[4]["narrow32"]  # refuted on the host: went up whole
    assert 27 in stats[5]["narrow32"]                  # relearned as 32-bit
    assert 27 not in stats[6]["narrow32"]              # refuted again


def test_upload_schedule_rejects_unknown_values():
    g = GpuProver(0, max_trace_len=1 << 10)
    try:
        for bad in (-1, 3, 99):
            assert native.lib().zk_prover_set_upload_schedule(g.handle, bad) == native.ZK_ERR_INVALID_ARG
        for ok in ("auto", "throughput", "latency"):
            g.set_upload_schedule(ok)
        with pytest.raises(KeyError):
            g.set_upload_schedule("fastest")
    finally:
        g.close()


def test_clock_column_derived_and_refuted(oracle):
    """The AIR clock (column 0 of an accepted trace holds 0 .. n-2 before its random last row): once learned, a
    host-resident trace's clock is neither uploaded nor transformed but derived (identity column + last-row
    correction) and checked by host threads.  A trace whose clock is not 0 .. n-2 (an invalid trace) must not be
    proved as the derived one: the host check refutes the derivation, the proof is redone from the caller's column
    and fails the AIR exactly as without the derivation; valid traces keep proving to the oracle's bytes."""
    trace, pub = workload_trace(ops_for_trace_len(14, "cipher"), seed=17)
    n = trace.shape[1]
    bad = trace.copy()
    bad[0, 1000] = [7, 0]  # clk[1000] = 7: not the clock
    other = trace.copy()
    other[0, n - 1] = [12345, 6789]  # another random last row: still a clock
    g = GpuProver(0, max_trace_len=n)
    try:
        derived = []
        for t in (trace, trace, other):
            proof, _, _, rc = g.prove(t, pub, ProofOptions())
            assert rc == 0
            assert proof == oracle.prove(t, oracle_pub(oracle, pub))[0]
            derived.append(g.upload_stats()["derived"])
        assert derived == [[], [0], [0]]
        _, _, _, rc = g.prove(bad, pub, ProofOptions(), allow_degree_error=True)
        assert rc == native.ZK_ERR_DEGREE
        proof, _, _, rc = g.prove(trace, pub, ProofOptions())  # not speculated again at this length
        assert rc == 0 and proof == oracle.prove(trace, oracle_pub(oracle, pub))[0]
        assert g.upload_stats()["derived"] == []
    finally:
        g.close()


def test_sparse_hint_learned_and_refuted(oracle):
    """The sparse hint (a host-resident trace's columns that the previous proof of the same length found sparse are
    taken as sparse from their last row, never uploaded, and checked by host threads during the proof): proofs of a
    trace, of the same trace again (hinted), of an edited trace the hint is wrong for (col 27 dense: the library must
    notice and redo the proof), and of the first trace once more -- each equal to the oracle's."""
    trace, pub = workload_trace(ops_for_trace_len(14, "cipher"), seed=15)
    n = trace.shape[1]
    edited = trace.copy()
    edited[27, 9] = [3, 1]     # dense now (no constraint reads s15: the trace still satisfies the AIR)
    edited[22, : n - 1] = 0    # sparse now
    g = GpuProver(0, max_trace_len=n)
    try:
        for t in (trace, trace, edited, edited, trace):
            proof, _, _, rc = g.prove(t, pub, ProofOptions())
            assert rc == 0
            oproof, _, _ = oracle.prove(t, oracle_pub(oracle, pub))
            assert proof == oproof
    finally:
        g.close()
