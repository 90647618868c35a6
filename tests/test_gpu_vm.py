"""The VM trace written on the GPU (zk_vm_trace_device, csrc/vm_gpu.hip) and vm::prove as one call (zk_vm_prove):
the device trace must equal the host VM's trace byte for byte (which the CPU tests pin to the oracle VM and to the
full-size pins' trace sha256), and zk_vm_prove's proof must equal the proof of the host trace."""
import hashlib
import random
import sys
from pathlib import Path

import numpy as np
import pytest

from zkvm_amd import native
from zkvm_amd.prover import GpuProver, Program, ProofOptions, ZkError, _hip, make_pub_inputs
from zkvm_amd.workloads import (LR_PROGRAM, LweParameters, cipher_mix_program, make_workload, ops_for_trace_len,
                                push_add_program)

sys.path.insert(0, str(Path(__file__).resolve().parent))
from golden_large import LARGE_CASES  # noqa: E402
from test_vm_parallel import random_program  # noqa: E402

pytestmark = pytest.mark.gpu


def device_trace(gpu, prog, w, last_row="given"):
    inp = Program.encode_inputs(w.public, w.secret, w.server_key)
    d, n, outs = prog.trace_device(gpu, inp, w.last_row if last_row == "given" else None)
    host = np.zeros((28, n, 2), dtype=np.uint64)
    import ctypes as C
    assert _hip().hipMemcpy(host.ctypes.data_as(C.c_void_p), C.c_void_p(d), host.nbytes, 2) == 0
    return host, outs


@pytest.fixture(scope="module")
def gpu():
    assert native.device_count() > 0, "no GPU visible"
    g = GpuProver(0, max_trace_len=1 << 16)
    yield g
    g.close()


@pytest.mark.parametrize("src", [LR_PROGRAM, push_add_program(100), cipher_mix_program(300)[0],
                                 ops_for_trace_len(14, "cipher"), ops_for_trace_len(16, "pushadd")],
                         ids=["lr", "pushadd100", "cipher300", "cipher_2p14", "pushadd_2p16"])
def test_device_trace_matches_host_vm(gpu, src):
    w = make_workload(src, seed=31)
    prog = Program(src)
    htrace, houts = prog.trace(w.public, w.secret, w.server_key, w.last_row)
    dtrace, douts = device_trace(gpu, prog, w)
    prog.close()
    assert douts == houts
    assert np.array_equal(dtrace, htrace)


@pytest.mark.parametrize("k", [1, 2, 3, 4])
def test_device_trace_other_lwe_sizes(gpu, k):
    """lwe_size 2..5 (the AIR's range; k = 4 is the default above): the templated device step per ciphertext
    width."""
    src = cipher_mix_program(40)[0]
    w = make_workload(src, seed=40 + k, params=LweParameters(k=k))
    prog = Program(src)
    htrace, houts = prog.trace(w.public, w.secret, w.server_key, w.last_row)
    dtrace, douts = device_trace(gpu, prog, w)
    prog.close()
    assert douts == houts and np.array_equal(dtrace, htrace)


def test_device_trace_random_programs(gpu):
    """The differential programs of test_vm_parallel (mostly valid, some failing): the same status and text as the
    host VM, and on success the same trace."""
    rnd = random.Random(4242)
    ok = 0
    for i in range(120):
        src = random_program(rnd)
        short = rnd.random() < 0.3
        w = make_workload(src or "push.1\n", seed=2000 + i, n_pub=rnd.randrange(0, 40) if short else None,
                          n_sec=rnd.randrange(0, 12) if short else None)
        try:
            prog = Program(src)
        except ZkError:
            continue
        try:
            htrace, houts = prog.trace(w.public, w.secret, w.server_key, w.last_row)
            hres = ("ok",)
        except ZkError as e:
            hres = ("err", e.code, str(e).split("] ", 1)[1])
        try:
            dtrace, douts = device_trace(gpu, prog, w)
            dres = ("ok",)
        except ZkError as e:
            dres = ("err", e.code, str(e).split(": ", 1)[1])
        prog.close()
        assert hres == dres, (src, hres, dres)
        if hres[0] == "ok":
            ok += 1
            assert douts == houts and np.array_equal(dtrace, htrace), src
    assert ok >= 15


@pytest.mark.parametrize("preprocess", ["1", "0"])
def test_vm_prove_equals_host_trace_proof(gpu, preprocess, monkeypatch):
    """zk_vm_prove (vm::prove with the trace written on the GPU) gives the proof of the host VM's trace, and the
    program hash / outputs of the reference's (hash, output, proof) -- with the program's preprocessed columns
    (default) and with every column generated and interpolated per proof (ZK_VM_PREPROCESS=0)."""
    monkeypatch.setenv("ZK_VM_PREPROCESS", preprocess)
    src = cipher_mix_program(200)[0]
    w = make_workload(src, seed=9)
    prog = Program(src)
    trace, outs = prog.trace(w.public, w.secret, w.server_key, w.last_row)
    pub = make_pub_inputs(prog.hash, outs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    ref, _, _, rc = gpu.prove(trace, pub, ProofOptions())
    assert rc == 0
    h, o, proof = prog.prove_device(gpu, Program.encode_inputs(w.public, w.secret, w.server_key), w.last_row)
    assert (h, o) == (prog.hash, outs) and proof == ref
    # a random last row (Processor::trace's thread_rng draw): a different, still valid proof
    from zkvm_amd.prover import verify
    _, o2, proof2 = prog.prove_device(gpu, Program.encode_inputs(w.public, w.secret, w.server_key), None)
    assert o2 == outs and proof2 != ref and verify(proof2, pub, 95) == (0, "")
    prog.close()


def test_vm_prove_reports_vm_errors(gpu):
    for src, msg in [("push.1\nadd\n", "add operation stack underflow"), ("read2\nread2\nread2\nread2\n",
                                                                          "read2 operation stack overflow"),
                     ("read\nread\n", "no more inputs to read")]:
        prog = Program(src)
        w = make_workload(src, seed=3, n_pub=1)
        host_err = None
        try:
            prog.trace(w.public, w.secret, w.server_key, w.last_row)
        except ZkError as e:
            host_err = (e.code, str(e).split("] ", 1)[1])
        assert host_err is not None and msg in host_err[1], (src, host_err)
        for pre in ("1", "0"):
            import os
            os.environ["ZK_VM_PREPROCESS"] = pre
            try:
                with pytest.raises(ZkError) as e:
                    prog.prove_device(gpu, Program.encode_inputs(w.public, w.secret, w.server_key), w.last_row)
            finally:
                os.environ.pop("ZK_VM_PREPROCESS", None)
            assert e.value.code == host_err[0] and str(e.value).endswith(host_err[1]), (src, pre, str(e.value))
        prog.close()


@pytest.mark.parametrize("log_n", sorted({c["log_n"] for c in LARGE_CASES if c["options"]["field_extension"] == 1
                                          and c["seed"] == 1000}))
def test_device_trace_full_size_pins(log_n, oracle):
    """configs[2] (2^20) and configs[3] (2^22): the device-written trace hashes to the pin's trace sha256 (the oracle
    VM's trace), and zk_vm_prove's proof equals the pinned proof byte for byte."""
    c = next(c for c in LARGE_CASES if c["log_n"] == log_n and c["seed"] == 1000
             and c["options"]["field_extension"] == 1)
    src = ops_for_trace_len(log_n, c["generator"])
    w = make_workload(src, seed=c["seed"])
    prog = Program(src)
    g = GpuProver(0, max_trace_len=1 << log_n)
    try:
        dtrace, _ = device_trace(g, prog, w)
        assert hashlib.sha256(dtrace.tobytes()).hexdigest() == c["trace_sha256"]
        del dtrace
        _, _, proof = prog.prove_device(g, Program.encode_inputs(w.public, w.secret, w.server_key), w.last_row)
    finally:
        g.close()
        prog.close()
    assert len(proof) == c["proof_len"] and hashlib.sha256(proof).hexdigest() == c["proof_sha256"]


def test_vm_prove_preprocessed_columns_across_provers_and_inputs(gpu):
    """The preprocessed columns are built once per (program, device, lwe_size, blowup) by whichever prover comes first
    and reused: a second prover, other inputs and a blowup-16 proof all give the host-trace proofs."""
    src = ops_for_trace_len(14, "cipher")
    prog = Program(src)
    g2 = GpuProver(0, max_trace_len=1 << 14, max_blowup=16)
    try:
        for seed, g, opts in [(1, gpu, ProofOptions()), (2, g2, ProofOptions()), (3, gpu, ProofOptions()),
                              (4, g2, ProofOptions(28, 16, 0, 1, 4, 63))]:
            w = make_workload(src, seed=seed)
            trace, outs = prog.trace(w.public, w.secret, w.server_key, w.last_row)
            pub = make_pub_inputs(prog.hash, outs, w.server_key.lwe_size(), w.server_key.parameters.delta)
            ref, _, _, rc = g.prove(trace, pub, opts)
            assert rc == 0
            _, _, proof = prog.prove_device(g, Program.encode_inputs(w.public, w.secret, w.server_key), w.last_row,
                                            opts)
            assert proof == ref, (seed, opts)
    finally:
        g2.close()
        prog.close()


def test_vm_prove_first_call_fails_then_succeeds(gpu):
    """The per-program preprocessed columns are built by the first zk_vm_prove call with that call's inputs: a first
    call the VM refuses (too few public inputs) must leave nothing cached, so the next call with valid inputs builds
    them afresh and proves exactly the host-trace proof."""
    src = cipher_mix_program(200)[0]
    w = make_workload(src, seed=21)
    short = make_workload(src, seed=21, n_pub=0)
    prog = Program(src)
    try:
        with pytest.raises(ZkError) as e:
            prog.prove_device(gpu, Program.encode_inputs(short.public, short.secret, short.server_key), w.last_row)
        assert "no more inputs to read" in str(e.value)
        trace, outs = prog.trace(w.public, w.secret, w.server_key, w.last_row)
        pub = make_pub_inputs(prog.hash, outs, w.server_key.lwe_size(), w.server_key.parameters.delta)
        ref, _, _, rc = gpu.prove(trace, pub, ProofOptions())
        assert rc == 0
        for _ in range(2):  # built by the first successful call, reused by the second
            _, _, proof = prog.prove_device(gpu, Program.encode_inputs(w.public, w.secret, w.server_key), w.last_row)
            assert proof == ref
    finally:
        prog.close()


def test_vm_prove_concurrent_first_calls():
    """Three provers on three host threads call zk_vm_prove at once on a freshly compiled program: one of them builds
    the program's preprocessed columns under the program lock while the others wait for it (the recursive-lock
    deadlock of round 4's first version would hang here); every proof equals the host-trace proof of its inputs."""
    import threading
    src = ops_for_trace_len(14, "cipher")
    prog = Program(src)
    provers = [GpuProver(0, max_trace_len=1 << 14) for _ in range(3)]
    try:
        ws = [make_workload(src, seed=60 + k) for k in range(3)]
        refs = []
        for k, w in enumerate(ws):
            trace, outs = prog.trace(w.public, w.secret, w.server_key, w.last_row)
            pub = make_pub_inputs(prog.hash, outs, w.server_key.lwe_size(), w.server_key.parameters.delta)
            ref, _, _, rc = provers[k].prove(trace, pub, ProofOptions())
            assert rc == 0
            refs.append(ref)
        prog.close()
        prog = Program(src)  # fresh: no device copy, no preprocessed columns yet
        got, errs = [None] * 3, []
        start = threading.Barrier(3)

        def run(k):
            try:
                start.wait()
                got[k] = prog.prove_device(provers[k], Program.encode_inputs(ws[k].public, ws[k].secret,
                                                                               ws[k].server_key), ws[k].last_row)[2]
            except BaseException as ex:  # re-raised below
                errs.append(ex)

        ths = [threading.Thread(target=run, args=(k,)) for k in range(3)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=90)
        assert not any(t.is_alive() for t in ths), "zk_vm_prove hung on the concurrent first call"
        assert not errs, errs
        assert got == refs
    finally:
        for g in provers:
            g.close()
        prog.close()
