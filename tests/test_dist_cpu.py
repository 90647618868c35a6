"""Multi-rank bench harness on CPU (2, 4 and 8 separate processes, no GPU, no torch in the ranks).

bench.py at N > 1 runs one process per GPU (torchrun's environment); each rank proves its own independent trace (weak
scaling, no data-path collective) and the timing is barrier-bracketed with the max taken over ranks.  The host side of
that runs over zkvm_amd.hostgroup (a TCP group; torch is never imported, so the library keeps its own HIP runtime and
RCCL).  Here the same code (bench.setup_dist / timed_loop / max_over_ranks) runs with a stand-in step of
rank-dependent duration: every rank must report the slowest rank's time.  The host group's collectives and its
zk_exchange_fn are checked byte for byte.
"""
import json
import os
import socket
import subprocess
import time
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent

WORKER = r'''
import json, os, sys, time
sys.path[:0] = [{root!r}, {pkg!r}]
mode = sys.argv[1]
if mode == "bench":
    import bench
    w, r, local, pg = bench.setup_dist(int(os.environ["WORLD_SIZE"]))
    calls = []
    def step():
        calls.append(1)
        time.sleep(0.03 * (r + 1))
    elapsed = bench.timed_loop(step, steps=4, warmup=2, pg=pg, local=local)
    ok = bench.all_ranks_true(pg, r != 1, local)
    out = {{"rank": r, "world": w, "elapsed": elapsed, "calls": len(calls), "all_true": ok,
            "torch": "torch" in sys.modules}}
    pg.close()
else:
    import ctypes as C
    from zkvm_amd import native
    from zkvm_amd.hostgroup import HostGroup
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    g = HostGroup.from_env(timeout=60)
    ag = g.all_gather(bytes([rank]) * (rank + 1))
    a2a = g.all_to_all([bytes([16 * rank + d]) * 3 for d in range(world)])
    big = g.all_gather(bytes([rank]) * (3 << 20))
    fn = g.exchange_fn()
    nb = 5
    send = (C.c_uint8 * (nb * world))(*[(16 * rank + d) & 255 for d in range(world) for _ in range(nb)])
    recv = (C.c_uint8 * (nb * world))()
    rc1 = fn(None, native.XCHG_ALL_TO_ALL, C.addressof(send), C.addressof(recv), nb)
    xa2a = list(recv)
    one = (C.c_uint8 * nb)(*[rank + 100] * nb)
    rc2 = fn(None, native.XCHG_ALL_GATHER, C.addressof(one), C.addressof(recv), nb)
    xag = list(recv)
    bad = fn(None, 7, C.addressof(one), C.addressof(recv), nb)
    uid = g.broadcast(b"id-from-rank-0" if rank == 0 else None)
    out = {{"ag": [list(x) for x in ag], "a2a": [list(x) for x in a2a], "big_ok": all(
        b == bytes([s]) * (3 << 20) for s, b in enumerate(big)), "x_a2a": xa2a, "x_ag": xag, "rc": [rc1, rc2],
        "bad_rc": bad, "uid": uid.decode(), "max": g.max(float(rank) * 1.5), "torch": "torch" in sys.modules}}
    g.close()
print("RESULT " + json.dumps(out), flush=True)
if os.environ.get("ZK_TEST_RESULT_DIR"):  # (under torchrun the ranks' stdout lines can interleave)
    with open(os.path.join(os.environ["ZK_TEST_RESULT_DIR"], "rank%d.json" % int(os.environ["RANK"])), "w") as f:
        json.dump(out, f)
'''


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_world(world, mode, tmp_path):
    """world processes with torchrun's environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT, run id)."""
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=str(ROOT), pkg=str(ROOT / "encrypt-zkvm_amd")))
    port, run_id = free_port(), f"t{os.getpid()}-{world}-{mode}"
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), TORCHELASTIC_RUN_ID=run_id, ZK_NUMA_BIND="0")
        procs.append(subprocess.Popen([sys.executable, str(script), mode], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=120)[0])
    finally:
        for p in procs:  # only the processes started here
            if p.poll() is None:
                p.kill()
                p.wait()
    res = []
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r}: {o}"
        res.append(json.loads(next(ln for ln in o.splitlines() if ln.startswith("RESULT "))[7:]))
    return res


@pytest.mark.parametrize("world", [2, 4, 8])
def test_timed_loop_max_over_ranks(world, tmp_path):
    res = sorted(run_world(world, "bench", tmp_path), key=lambda x: x["rank"])
    times = [x["elapsed"] for x in res]
    assert all(x["calls"] == 6 for x in res)                    # warmup 2 + steps 4 on every rank
    assert max(times) - min(times) < 1e-9                        # every rank reports the same (max) time
    assert times[0] >= 4 * 0.03 * world * 0.95                   # ... which is the slowest rank's
    assert all(x["all_true"] is False for x in res)             # rank 1's False reaches every rank
    assert not any(x["torch"] for x in res)                      # the bench process never imports torch


@pytest.mark.parametrize("world", [2, 3])
def test_host_group_collectives(world, tmp_path):
    res = run_world(world, "group", tmp_path)
    nb = 5
    for r, x in enumerate(res):
        assert x["ag"] == [[s] * (s + 1) for s in range(world)]
        assert x["a2a"] == [[16 * s + r] * 3 for s in range(world)]
        assert x["big_ok"]
        assert x["rc"] == [0, 0] and x["bad_rc"] != 0
        # the zk_exchange_fn layout: all-to-all chunk s of rank r's recv is chunk r of rank s's send
        assert x["x_a2a"] == [16 * s + r for s in range(world) for _ in range(nb)]
        assert x["x_ag"] == [100 + s for s in range(world) for _ in range(nb)]
        assert x["uid"] == "id-from-rank-0"
        assert x["max"] == 1.5 * (world - 1)
        assert not x["torch"]


def test_under_torchrun(tmp_path):
    """The driver's launch form: torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1
    --master-port P.  The launcher's agent holds MASTER_PORT (its TCPStore); the torch-free ranks meet through the
    host group's rendezvous file instead and report the same max-over-ranks time."""
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=str(ROOT), pkg=str(ROOT / "encrypt-zkvm_amd")))
    env = dict(os.environ, ZK_NUMA_BIND="0", ZK_TEST_RESULT_DIR=str(tmp_path))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(script), "bench"],
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = [json.loads((tmp_path / f"rank{k}.json").read_text()) for k in range(2)]
    assert sorted(x["rank"] for x in res) == [0, 1]
    assert res[0]["elapsed"] == res[1]["elapsed"] and not any(x["torch"] for x in res)


def test_host_group_peer_death_is_an_error_not_a_hang(tmp_path):
    """A rank that dies mid-run (a crashed or killed GPU process) makes the others' next collective raise
    ConnectionError promptly instead of waiting forever (the bench's watchdog is the second line)."""
    code = r'''
import os, sys, time, json
sys.path[:0] = [{pkg!r}]
from zkvm_amd.hostgroup import HostGroup
rank = int(os.environ["RANK"])
g = HostGroup.from_env(timeout=60)
g.barrier()
if rank == 1:
    os._exit(0)
t0 = time.monotonic()
try:
    g.all_gather(b"x" * 1024)
    print("RESULT " + json.dumps({{"raised": False}}))
except ConnectionError as e:
    print("RESULT " + json.dumps({{"raised": True, "s": time.monotonic() - t0}}))
'''.format(pkg=str(ROOT / "encrypt-zkvm_amd"))
    script = tmp_path / "die.py"
    script.write_text(code)
    port = free_port()
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(os.environ, RANK=str(r), WORLD_SIZE="2",
                                                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                                                                       TORCHELASTIC_RUN_ID=f"die{os.getpid()}"),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    out = procs[0].communicate(timeout=60)[0]
    procs[1].communicate(timeout=60)
    res = json.loads(next(ln for ln in out.splitlines() if ln.startswith("RESULT "))[7:])
    assert res["raised"] and res["s"] < 10, out


def test_workload_seeds_differ_per_rank():
    """Each rank proves an independent trace: bench seeds the generator with 1000 + rank."""
    sys.path.insert(0, str(ROOT / "encrypt-zkvm_amd"))
    from zkvm_amd.workloads import cipher_mix_program, make_workload
    src = cipher_mix_program(4)[0]
    a, b = make_workload(src, seed=1000), make_workload(src, seed=1001)
    assert a.secret != b.secret and a.last_row != b.last_row


def test_numa_cpulist_parsing():
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import bench
    assert bench._cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert bench._cpulist("") == set()
    # no GPU here: the binding finds no device and leaves the affinity alone
    before = os.sched_getaffinity(0)
    assert bench.bind_to_gpu_numa_node(0) is None
    assert os.sched_getaffinity(0) == before


def test_host_group_refuses_an_address_of_another_host():
    """every rank of the torch-free host group runs on the MASTER_ADDR host; another host's address fails
    at once with the reason instead of retrying to the deadline."""
    import time
    from zkvm_amd.hostgroup import HostGroup
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match="not an address of this host"):
        HostGroup(1, 2, addr="192.0.2.1", rdzv_key="no-such-run", timeout=30)  # TEST-NET-1: never local
    assert time.monotonic() - t0 < 5


def test_host_group_skips_a_stale_rendezvous_port(tmp_path):
    """A rendezvous file left by an earlier run can name a port that now belongs to a listener that accepts but never
    answers: the connecting rank gives up on it within seconds (the hub greets first) and reads the file again."""
    import threading
    from zkvm_amd import hostgroup
    from zkvm_amd.hostgroup import HostGroup
    key = f"stale-{os.getpid()}"
    silent = socket.create_server(("127.0.0.1", 0))  # accepts (backlog), never replies
    path = hostgroup._rdzv_file("127.0.0.1", key)
    with open(path, "w") as f:
        f.write(f"{silent.getsockname()[1]} deadbeef00000000\n")
    out = {}

    def rank1():
        try:
            g = HostGroup(1, 2, addr="127.0.0.1", rdzv_key=key, timeout=60)
            out[1] = g.all_gather(b"r1")
            g.close()
        except Exception as e:  # reported below
            out[1] = e

    t = threading.Thread(target=rank1)
    t.start()
    time.sleep(1.0)  # rank 1 has read the stale file and sits on the silent port
    g0 = HostGroup(0, 2, addr="127.0.0.1", rdzv_key=key, timeout=60)
    got0 = g0.all_gather(b"r0")
    g0.close()
    t.join(60)
    silent.close()
    assert got0 == [b"r0", b"r1"] and out[1] == [b"r0", b"r1"], out
