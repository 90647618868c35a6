"""The sharded prover with one rank per PROCESS (zk_comm_create_host + a TCP host group), as an RCCL job runs it.

The loopback tests (tests/test_sharded.py) drive every rank from one process; here `world` separate processes on
the one test GPU each hold a single rank-sized prover, so every rank-dependent branch of shard.hip (coset ownership,
the openings each rank serves, FRI layers >= 1 on rank 0, the per-process transcript) runs as in a multi-GPU job --
only the transport differs (zkvm_amd.hostgroup over 127.0.0.1 instead of RCCL over xGMI).  The CPU tests check the
exchange callback's chunk order at world 2, and the communicator's argument checks.  No process imports torch: every
rank runs on the HIP runtime the library links (checked in the rank records).
"""
import ctypes as C
import json
import socket
import subprocess
import sys
from pathlib import Path

import pytest

from zkvm_amd import native

WORKER = Path(__file__).resolve().parent / "sharded_worker.py"


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return str(s.getsockname()[1])


def run_ranks(world, out, mode="prove", timeout=240, env=None):
    port = free_port()
    procs = [subprocess.Popen([sys.executable, "-u", str(WORKER), str(r), str(world), port, str(out), mode],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
             for r in range(world)]
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:  # only the processes started here
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{logs[r] if r < len(logs) else ''}"
    return [json.loads((out / f"rank{r}.json").read_text()) for r in range(world)]


def test_host_exchange_callback_world2(tmp_path):
    res = run_ranks(2, tmp_path, "selftest", timeout=120)
    nb, world = 5, 2
    for r, x in enumerate(res):
        # all-to-all: chunk s of rank r's recv is chunk r of rank s's send (value 16 s + r)
        assert x["a2a"] == [16 * s + r for s in range(world) for _ in range(nb)]
        assert x["ag"] == [100 + s for s in range(world) for _ in range(nb)]
        assert x["bad_op_rc"] != 0


def test_host_comm_argument_checks():
    L = native.lib()
    comm = C.c_void_p()
    fn = native.EXCHANGE_FN(lambda *a: 0)
    assert L.zk_comm_create_host(0, 3, fn, None, C.byref(comm)) == native.ZK_ERR_INVALID_ARG
    assert L.zk_comm_create_host(2, 2, fn, None, C.byref(comm)) == native.ZK_ERR_INVALID_ARG
    assert L.zk_comm_create_host(0, 2, native.EXCHANGE_FN(), None, C.byref(comm)) == native.ZK_ERR_INVALID_ARG
    assert L.zk_comm_create_host(1, 4, fn, None, C.byref(comm)) == native.ZK_OK
    L.zk_comm_destroy(comm)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_one_rank_per_process(tmp_path, world):
    res = run_ranks(world, tmp_path)
    for x in res:
        rt = x.pop("runtime")
        assert isinstance(rt["hip_runtime"], str) and not rt["torch_loaded_first"], rt
    names = sorted(res[0])
    assert len(names) >= 3 and all(sorted(x) == names for x in res)
    for name in names:
        want = res[0][name]["want"]  # golden sha, or rank 0's single-GPU proof for the generated traces
        assert want, name
        for r, x in enumerate(res):
            assert x[name]["sha256"] == want, (name, r)


# full-size pinned configs with every rank in its own process: configs[2] (2^20) over 8 ranks, configs[4] (2^20, quadratic
# extension, 128 bits) over 4, configs[3] (2^22) over 8 -- the north_star's sharded proof, with TCP host exchanges in place of RCCL;
# each rank regenerates the trace with the product VM (2 threads: the box's CPU share is split between the processes)
# and checks the proof against the oracle's pin and both verifiers
FULL_SIZE_MP = [("c2_cipher_2p20", 8), ("c4_cipher_2p20_quad", 4), ("c3_cipher_2p22", 8)]


@pytest.mark.gpu
@pytest.mark.parametrize("name,world", FULL_SIZE_MP, ids=[f"{n}-w{w}" for n, w in FULL_SIZE_MP])
def test_sharded_one_rank_per_process_full_size(oracle, tmp_path, name, world):
    import os  # (the oracle fixture builds the checker library once, before the ranks start)
    res = run_ranks(world, tmp_path, f"large:{name}", timeout=280, env={**os.environ, "ZK_VM_THREADS": "2"})
    assert all(x[name]["sha256"] == x[name]["want"] for x in res)
