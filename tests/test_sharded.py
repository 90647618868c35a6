"""Coset-sharded proving (zk_prove_sharded) on one GPU through the loopback
communicator: every world size gives proof bytes identical to the golden (oracle) proofs and to the
single-GPU prover.  The RCCL communicator runs the same code with one rank per process; its only
difference is the transport of the all-to-all / all-gather steps."""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

from zkvm_amd import native
from zkvm_amd.prover import GpuProver, ProofOptions, make_pub_inputs
from zkvm_amd.sharded import ShardedProver

GOLD = Path(__file__).resolve().parent / "golden"
CASES = [c for c in json.loads((GOLD / "cases.json").read_text())["cases"] if c["options"]["blowup"] == 8]


def ints(hs):
    return [int(h, 16) for h in hs]


def case_inputs(c):
    trace = np.load(GOLD / f"{c['name']}.trace.npy", allow_pickle=False)
    proof = (GOLD / f"{c['name']}.proof").read_bytes()
    pub = make_pub_inputs(ints(c["program_hash"]), ints(c["stack_outputs"]), c["lwe_size"], c["delta"])
    o = c["options"]
    opts = ProofOptions(o["num_queries"], o["blowup"], o["grinding"], o["field_extension"], o["fri_folding"],
                        o["fri_rem_max_deg"])
    return trace, proof, pub, opts


def fits(c, world):
    n, fold = c["trace_len"], c["options"]["fri_folding"]
    return n // fold >= 8 * world and n // world >= 8


FITTING = [(c, w) for c in CASES for w in (1, 2, 4, 8) if fits(c, w)]
TOO_SHORT = [(c, w) for c in CASES for w in (1, 2, 4, 8) if not fits(c, w)]


@pytest.mark.gpu
@pytest.mark.parametrize("c,world", FITTING, ids=[f"{c['name']}-w{w}" for c, w in FITTING])
def test_sharded_matches_golden(c, world):
    trace, proof, pub, opts = case_inputs(c)
    sp = ShardedProver.loopback(world, max_trace_len=trace.shape[1])
    try:
        got, rec = sp.prove(trace, pub, opts, record=True)
    finally:
        sp.close()
    assert bytes(rec.trace_root).hex() == c["trace_root"]
    assert bytes(rec.constraint_root).hex() == c["constraint_root"]
    assert [bytes(rec.fri_roots[i]).hex() for i in range(rec.num_fri_layers)] == c["fri_roots"]
    assert got == proof


@pytest.mark.gpu
@pytest.mark.parametrize("c,world", TOO_SHORT, ids=[f"{c['name']}-w{w}" for c, w in TOO_SHORT])
def test_sharded_refuses_too_short_trace(c, world):
    """A trace whose FRI layer 1 or coset slices are smaller than the rank count is refused up front
    (ZK_ERR_INVALID_ARG), never proved with a wrong split."""
    trace, _, pub, opts = case_inputs(c)
    sp = ShardedProver.loopback(world, max_trace_len=trace.shape[1])
    try:
        with pytest.raises(native.ZkError) as e:
            sp.prove(trace, pub, opts)
    finally:
        sp.close()
    assert e.value.code == native.ZK_ERR_INVALID_ARG and "too short" in str(e.value)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
@pytest.mark.parametrize("ext", [1, 2])
def test_sharded_matches_single_gpu_2_14(world, ext):
    from zkvm_amd.prover import vm_trace
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    src = ops_for_trace_len(14, "cipher")
    w = make_workload(src, seed=21)
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    opts = ProofOptions(field_extension=ext)
    g = GpuProver(0, max_trace_len=trace.shape[1])
    try:
        single, _, _, rc = g.prove(trace, pub, opts)
    finally:
        g.close()
    assert rc == 0
    sp = ShardedProver.loopback(world, max_trace_len=trace.shape[1])
    try:
        got, _ = sp.prove(trace, pub, opts)
    finally:
        sp.close()
    assert hashlib.sha256(got).hexdigest() == hashlib.sha256(single).hexdigest()


@pytest.mark.gpu
@pytest.mark.parametrize("fold,rem,ext", [(2, 127, 1), (4, 127, 2), (16, 127, 1), (16, 63, 2), (8, 31, 2)])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_fri_layer1_folds_2_14(world, fold, rem, ext):
    """Sharded FRI layer 1 (taken when the prover has two or more layers and layer 1 holds >= 8 points per rank) at
    every folding factor, both extensions and the in-place / staged gathered layer: byte-identical to one GPU."""
    from zkvm_amd.prover import vm_trace
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    src = ops_for_trace_len(14, "pushadd")
    w = make_workload(src, seed=5 + fold)
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    opts = ProofOptions(field_extension=ext, fri_folding_factor=fold, fri_remainder_max_degree=rem)
    g = GpuProver(0, max_trace_len=trace.shape[1])
    try:
        single, _, _, rc = g.prove(trace, pub, opts)
    finally:
        g.close()
    assert rc == 0
    sp = ShardedProver.loopback(world, max_trace_len=trace.shape[1])
    try:
        got, _ = sp.prove(trace, pub, opts)
    finally:
        sp.close()
    assert got == single


@pytest.mark.gpu
def test_sharded_rccl_world1_and_device_trace():
    """The RCCL communicator (one rank on this GPU) and the device-resident trace path."""
    c = next(c for c in CASES if c["name"] == "cipher20")
    trace, proof, pub, opts = case_inputs(c)
    sp = ShardedProver.rccl(0, 1, ShardedProver.unique_id(), 0, trace.shape[1])
    try:
        got, _ = sp.prove(trace, pub, opts)
        assert got == proof
        n = sp.upload_trace(trace)
        got2, _ = sp.prove(None, pub, opts, n=n)
        assert got2 == proof
    finally:
        sp.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_device_trace(world):
    """Every rank's device trace buffer already holds the trace (zk_prove_sharded with trace = NULL): each rank
    interpolates its slice of the columns from it; same proof bytes as from the host trace."""
    c = next(c for c in CASES if c["name"] == "cipher20")
    trace, proof, pub, opts = case_inputs(c)
    sp = ShardedProver.loopback(world, max_trace_len=trace.shape[1])
    try:
        n = sp.upload_trace(trace)
        got, _ = sp.prove(None, pub, opts, n=n)
        assert got == proof
        got2, _ = sp.prove(trace, pub, opts)
        assert got2 == proof
    finally:
        sp.close()


def test_sharded_rejects_bad_world():
    import ctypes as C
    comm = C.c_void_p()
    assert native.lib().zk_comm_create_loopback(3, C.byref(comm)) == native.ZK_ERR_INVALID_ARG


# ---------------------------------------------------------------- full-size pins, sharded
from golden_large import LARGE_CASES, check_large_proof, large_inputs  # noqa: E402
@pytest.mark.gpu
@pytest.mark.parametrize("log_n,world,ext,pre", [(14, 2, 1, True), (14, 8, 2, True), (16, 8, 1, True), (16, 4, 2, True),
                                                 (16, 1, 1, True), (16, 8, 1, False), (14, 2, 2, False)])
def test_sharded_vm_prove(log_n, world, ext, pre, monkeypatch):
    """vm::prove sharded (zk_vm_prove_sharded): every loopback rank writes the trace on its own device buffer, then
    one sharded proof over them -- with the per-program preprocessed columns of each rank's own cosets (the default;
    pre=False: every column from the device trace, ZK_VM_PREPROCESS=0), and the assertion terms split by coefficient
    range.  The bytes equal the single-GPU proof of the host trace; a second call reuses the preprocessed columns."""
    if not pre:
        monkeypatch.setenv("ZK_VM_PREPROCESS", "0")
    from zkvm_amd.prover import Program
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    src = ops_for_trace_len(log_n, "cipher")
    w = make_workload(src, seed=22 + log_n)
    prog = Program(src)
    trace, outputs = prog.trace(w.public, w.secret, w.server_key, w.last_row)
    pub = make_pub_inputs(prog.hash, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    opts = ProofOptions(field_extension=ext)
    g = GpuProver(0, max_trace_len=trace.shape[1])
    try:
        single, _, _, rc = g.prove(trace, pub, opts)
    finally:
        g.close()
    assert rc == 0
    inp = Program.encode_inputs(w.public, w.secret, w.server_key)
    sp = ShardedProver.loopback(world, max_trace_len=trace.shape[1])
    try:
        h, outs, got = sp.prove_program(prog, inp, w.last_row, opts)
        assert h == list(prog.hash) and outs == list(outputs)
        assert sp.prove_program(prog, inp, w.last_row, opts)[2] == got
        with pytest.raises(native.ZkError):  # the last row must be given: every rank writes the same trace
            native.check(native.lib().zk_vm_prove_sharded(sp.comm, None, 0, prog.handle, None, 0, None, 0, 4, 1,
                                                          None, None, None, None, None, None))
    finally:
        sp.close()
        prog.close()
    assert hashlib.sha256(got).hexdigest() == hashlib.sha256(single).hexdigest()


# (case, world): every loopback rank holds its own rank-sized prover (zk_prover_create_shard) on the one test GPU:
# 2^22 at world 8 is 8 x ~12.6 GB
LARGE_SHARDED = [(c, w) for c in LARGE_CASES for w in ((8,) if c["log_n"] <= 20 else (2, 8))]


@pytest.mark.gpu
@pytest.mark.parametrize("c,world", LARGE_SHARDED, ids=[f"{c['name']}-w{w}" for c, w in LARGE_SHARDED])
def test_sharded_full_size_matches_oracle_pin(oracle, c, world):
    """The coset-sharded prover (loopback ranks) on the full-size configs: proof bytes equal the oracle's pin."""
    ht, trace, pub, opts = large_inputs(c)
    sp = ShardedProver.loopback(world, max_trace_len=trace.shape[1])
    try:
        proof, rec = sp.prove(trace, pub, opts, record=True)
    finally:
        sp.close()
        ht.close()
    check_large_proof(c, proof, rec, pub, oracle)


@pytest.mark.gpu
def test_shard_prover_refuses_single_gpu_calls():
    """A prover sized for one rank of a sharded proof holds 1/world of the LDE domain: the single-GPU entry
    points refuse it, and zk_prove_sharded refuses it for another world size."""
    import ctypes as C
    from zkvm_amd.prover import GpuProver
    c = CASES[0]
    trace, proof, pub, opts = case_inputs(c)
    n = trace.shape[1]
    L = native.lib()
    h = C.c_void_p()
    native.check(L.zk_prover_create_shard(0, n, 4, C.byref(h)))
    try:
        g = GpuProver.__new__(GpuProver)
        g.handle, g.max_trace_len, g.device = h, n, 0
        with pytest.raises(native.ZkError) as e:
            g.prove(trace, pub, opts)
        assert e.value.code == native.ZK_ERR_INVALID_ARG and "sharded" in str(e.value)
        g.handle = None  # the handle is destroyed below, not by the wrapper
        comm = C.c_void_p()
        native.check(L.zk_comm_create_loopback(2, C.byref(comm)))
        arr = (C.c_void_p * 2)(h.value, h.value)
        plen = C.c_size_t(1 << 20)
        buf = C.create_string_buffer(1 << 20)
        opt = opts.to_c()
        rc = L.zk_prove_sharded(comm, arr, 2, trace.ctypes.data, n, C.byref(opt), C.byref(pub), buf, C.byref(plen), None)
        assert rc == native.ZK_ERR_INVALID_ARG
        L.zk_comm_destroy(comm)
    finally:
        L.zk_prover_destroy(h)



@pytest.mark.gpu
@pytest.mark.parametrize("world,ext", [(2, 1), (8, 1), (4, 2)])
def test_sharded_host_column_hints(world, ext):
    """Host-trace sharded proofs with the column hints of the previous sharded proof (shard.hip S2): the sparse columns
    and the AIR clock are taken from the last row (not uploaded, interpolated or all-gathered) and checked by every
    rank's host threads over its row range.  A trace the hints are wrong for (a hinted sparse column made dense in a
    column no constraint reads) is refuted on every rank and proved again from every column; a trace whose clock is
    not 0 .. n-2 is not proved as the derived one (it fails the AIR as without the hints).  Every proof equals the
    single-GPU prover's."""
    from zkvm_amd.prover import vm_trace
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    src = ops_for_trace_len(16, "cipher")
    w = make_workload(src, seed=81 + world)
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    n = trace.shape[1]
    dense = trace.copy()
    dense[27, 9] = [3, 1]        # s15 (read by no constraint): dense now
    other = trace.copy()
    other[0, n - 1] = [4242, 17]  # another last row: still a clock
    bad = trace.copy()
    bad[0, 1000] = [7, 0]        # not a clock
    opts = ProofOptions(field_extension=ext)
    g = GpuProver(0, max_trace_len=n)
    sp = ShardedProver.loopback(world, max_trace_len=n)
    try:
        for t in (trace, trace, trace, dense, dense, other, trace):
            want, _, _, rc = g.prove(t, pub, opts)
            assert rc == 0
            got, _ = sp.prove(t, pub, opts)
            assert hashlib.sha256(got).hexdigest() == hashlib.sha256(want).hexdigest()
        with pytest.raises(native.ZkError) as e:
            sp.prove(bad, pub, opts)
        assert e.value.code == native.ZK_ERR_DEGREE
        got, _ = sp.prove(trace, pub, opts)  # (the clock is not speculated again at this length)
        assert got == g.prove(trace, pub, opts)[0]
    finally:
        sp.close()
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_trace_split_and_measurement_mode_keep_the_bytes(world):
    """Round 6: the trace interpolation of device-resident traces splits any number of columns round robin and
    interpolates the rest on every rank (zk_comm_set_trace_split), and the exchanges overlap compute on a stream of
    their own; the measurement mode serialises everything on one stream and logs the schedule.  Every split, both
    modes and the vm::prove path give the single-GPU proof, and the schedule log accounts for every exchange."""
    from zkvm_amd.prover import Program, vm_trace
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    src = ops_for_trace_len(16, "cipher")
    w = make_workload(src, seed=61)
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    n = trace.shape[1]
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    g = GpuProver(0, max_trace_len=n)
    try:
        want = g.prove_host(trace, pub, ProofOptions())[0]
    finally:
        g.close()
    prog = Program(src)
    inp = Program.encode_inputs(w.public, w.secret, w.server_key)
    sp = ShardedProver.loopback(world, max_trace_len=n)
    try:
        for measure in (False, True):
            sp.set_measure(measure)
            for rep in (-1, 0, 3, 28):
                sp.set_trace_split(rep)
                sp.upload_trace(trace)
                assert sp.prove(None, pub, ProofOptions(), n=n)[0] == want, (measure, rep)
                sc = sp.schedule()
                starts = [e for e in sc["entries"] if "start" in e]
                waits = {e["wait"] for e in sc["entries"] if "wait" in e}
                assert sc["world"] == world and sc["measure"] == measure
                assert {e["start"] for e in starts} == waits  # every exchange started is waited for
                assert all(e["seg_ms"] >= 0 for e in sc["entries"] if "seg_ms" in e)
                assert sp.prove_program(prog, inp, w.last_row)[2] == want, (measure, rep)
            assert sp.prove(trace, pub, ProofOptions())[0] == want  # host trace: every column split
        stats = sp.exchange_stats(exposed=True)
        assert stats and all(len(v) == 4 and v[3] >= 0 for v in stats.values())
    finally:
        sp.close()
        prog.close()
