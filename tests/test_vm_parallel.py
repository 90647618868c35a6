"""The product VM (csrc/vm.cpp) in the reference's two steps: zk_program_compile (Program::compile,
vm/src/program/mod.rs:37-131, keeping the chiplet's sponge states) and zk_program_trace (Processor::run + trace,
vm/src/processor/mod.rs:61-95: a sequential stack pass, then threaded row writes).  CPU tests against the oracle's
VM (oracle/vm.c) and the full-size pins the oracle produced (tests/golden/large, tools/gen_golden_large.py).
"""
import hashlib
import json
import os
import random
from pathlib import Path

import numpy as np
import pytest

from zkvm_amd import native
from zkvm_amd.prover import Program, ZkError, vm_trace
from zkvm_amd.workloads import ServerKey, cipher_mix_program, make_workload, ops_for_trace_len

LARGE = Path(__file__).resolve().parent / "golden" / "large" / "cases.json"
LARGE_CASES = json.loads(LARGE.read_text())["cases"] if LARGE.exists() else []


def ints(xs):
    return [int(x, 16) for x in xs]


@pytest.mark.parametrize("log_n", sorted({c["log_n"] for c in LARGE_CASES}))
def test_full_size_traces_match_oracle_pins(log_n):
    """configs[2] / [4] (2^20) and configs[3] (2^22): the product VM's trace, program hash and stack outputs equal
    the oracle VM's (sha256 of the 28 x n trace the oracle proved in tools/gen_golden_large.py)."""
    c = next(c for c in LARGE_CASES if c["log_n"] == log_n)
    src = ops_for_trace_len(log_n, c["generator"])
    w = make_workload(src, seed=c["seed"])
    prog = Program(src)
    assert prog.trace_len == 1 << log_n and prog.hash == ints(c["program_hash"])
    trace, outputs = prog.trace(w.public, w.secret, w.server_key, w.last_row)
    assert hashlib.sha256(trace.tobytes()).hexdigest() == c["trace_sha256"]
    assert outputs == ints(c["stack_outputs"])
    prog.close()


def test_thread_counts_give_identical_traces(oracle, monkeypatch):
    src = ops_for_trace_len(16, "cipher")
    w = make_workload(src, seed=5)
    prog = Program(src)
    got = []
    for t in ("1", "3", "8", "16"):
        monkeypatch.setenv("ZK_VM_THREADS", t)
        got.append(prog.trace(w.public, w.secret, w.server_key, w.last_row)[0])
    assert all(np.array_equal(g, got[0]) for g in got[1:])
    codes, values, h = oracle.program_compile(src)
    otrace, outs = oracle.processor_trace(codes, values, w.public, w.secret, 5, 16, w.last_row)
    assert np.array_equal(got[0], otrace) and h == prog.hash


def test_compiled_program_traces_many_inputs(oracle):
    """One compile, several runs on different inputs (the sponge columns are reused): each run equals the
    oracle's trace of the same inputs."""
    src = cipher_mix_program(40)[0]
    prog = Program(src)
    codes, values, _ = oracle.program_compile(src)
    for seed in range(3):
        w = make_workload(src, seed=50 + seed)
        trace, outs = prog.trace(w.public, w.secret, w.server_key, w.last_row)
        otrace, oouts = oracle.processor_trace(codes, values, w.public, w.secret, 5, 16, w.last_row)
        assert np.array_equal(trace, otrace) and outs == oouts


TOKENS = ["push.1", "push.0", "push.255", "push.256", "push.", "push.x", "push.+7", "read", "read2", "add", "add2",
          "mul", "smul", "sadd", "noop", "# c", "", "push.3.4", "add.1", "READ"]
BLOCK = ["read2", "read", "smul", "add2", "read", "sadd", "push.3", "push.5", "mul", "add", "read", "smul"]


def random_program(rnd: random.Random) -> str:
    lines = ["read2", "read", "smul"] if rnd.random() < 0.5 else []
    structured = bool(lines)
    for k in range(rnd.randrange(0, 120)):
        lines.append(BLOCK[k % len(BLOCK)] if structured and rnd.random() < 0.95 else rnd.choice(TOKENS))
    return "\n".join(lines) + "\n"


def test_random_programs_match_oracle_vm(oracle):
    """Differential: random (mostly valid, some malformed) programs and input vectors through the product VM and
    the oracle VM -- the same status, the same error text, and on success the same trace, outputs and hash."""
    rnd = random.Random(20261017)
    ran = 0
    for i in range(200):
        src = random_program(rnd)
        # enough inputs for every read most of the time, too few now and then
        short = rnd.random() < 0.3
        w = make_workload(src or "push.1\n", seed=i, n_pub=rnd.randrange(0, 40) if short else None,
                          n_sec=rnd.randrange(0, 12) if short else None)
        try:
            codes, values, h = oracle.program_compile(src)
            otrace, oouts = oracle.processor_trace(codes, values, w.public, w.secret, 5, 16, w.last_row)
            ores = ("ok", otrace, oouts, h)
        except oracle.OracleError as e:
            ores = ("err", e.code, str(e))
        try:
            trace, outs, ph = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
            res = ("ok", trace, outs, ph)
        except ZkError as e:
            res = ("err", e.code, str(e).split("] ", 1)[1])
        assert res[0] == ores[0], (src, res[:1], ores[1:] if ores[0] == "err" else None)
        if res[0] == "ok":
            ran += 1
            assert np.array_equal(res[1], ores[1]) and res[2] == ores[2] and res[3] == ores[3], src
        else:
            assert res[1] == ores[1] and res[2] == ores[2], (src, res, ores)
    assert ran >= 15


def test_program_errors_surface():
    with pytest.raises(ZkError) as e:
        Program("push.1\nfoo\n")
    assert e.value.code == native.ZK_ERR_PROGRAM and "instruction foo is invalid" in str(e.value)
    prog = Program("add\n")
    with pytest.raises(ZkError) as e:
        prog.trace([], [], ServerKey(seed=0), [1] * 28)
    assert e.value.code == native.ZK_ERR_STACK and "stack underflow" in str(e.value)


def test_stack_pass_states_match_trace_rows():
    """The host stack pass behind the device trace generator (vm.cpp stack_pass: bottom-first stack, one store per
    push) against the rows the reference-shaped VM writes: state c equals row c*stride - 1 (registers, depth), the
    outputs agree, and a failing run reports the same status and text."""
    rnd = random.Random(77)
    checked = 0
    for i in range(160):
        src = random_program(rnd)
        short = rnd.random() < 0.3
        w = make_workload(src or "push.1\n", seed=1000 + i, n_pub=rnd.randrange(0, 40) if short else None,
                          n_sec=rnd.randrange(0, 12) if short else None)
        try:
            prog = Program(src)
        except ZkError:
            continue
        try:
            trace, outs = prog.trace(w.public, w.secret, w.server_key, w.last_row)
        except ZkError as e:
            with pytest.raises(ZkError) as e2:
                prog.stack_states(w.public, w.secret, w.server_key, 8, 4)
            assert e2.value.code == e.code and str(e2.value).split("] ", 1)[1] == str(e).split("] ", 1)[1]
            prog.close()
            continue
        n = trace.shape[1]
        for stride in (8, 16, 64):
            if stride > n:
                continue
            count = n // stride
            states, souts = prog.stack_states(w.public, w.secret, w.server_key, stride, count)
            assert souts == outs
            assert not states[0].any()
            rows = np.arange(1, count) * stride - 1
            assert np.array_equal(states[1:, :16, :], trace[12:28, rows, :].transpose(1, 0, 2))
            assert np.array_equal(states[1:, 16, 0] & 0xFFFFFFFF, trace[11, rows, 0])
        prog.close()
        checked += 1
    assert checked >= 20


def test_stack_pass_full_size_pin():
    """configs[2]'s 2^20 trace: the stack pass's states every 64 rows (what the device generator uploads) equal the
    rows of the pinned trace."""
    c = next(c for c in LARGE_CASES if c["log_n"] == 20)
    src = ops_for_trace_len(20, c["generator"])
    w = make_workload(src, seed=c["seed"])
    prog = Program(src)
    trace, outs = prog.trace(w.public, w.secret, w.server_key, w.last_row)
    assert hashlib.sha256(trace.tobytes()).hexdigest() == c["trace_sha256"]
    states, souts = prog.stack_states(w.public, w.secret, w.server_key, 64, (1 << 20) // 64)
    rows = np.arange(1, (1 << 20) // 64) * 64 - 1
    assert souts == outs
    assert np.array_equal(states[1:, :16, :], trace[12:28, rows, :].transpose(1, 0, 2))
    assert np.array_equal(states[1:, 16, 0] & 0xFFFFFFFF, trace[11, rows, 0])
    prog.close()
