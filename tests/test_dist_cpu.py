"""Multi-rank bench harness on CPU (gloo, world_size 2).

bench.py at N > 1 runs one process per GPU; each rank proves its own independent trace (weak
scaling, no data-path collective) and the timing is barrier-bracketed with the max taken over
ranks.  Here the same code (bench.setup_dist / timed_loop / max_over_ranks) runs under gloo with
a stand-in step of rank-dependent duration: every rank must report the slowest rank's time.
"""
import os
import socket
import sys
import time
from pathlib import Path

import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, str(ROOT))
    import bench
    w, r, local, pg = bench.setup_dist(world)
    assert (w, r) == (world, rank) and pg is not None
    calls = []

    def step():
        calls.append(1)
        time.sleep(0.03 * (rank + 1))

    elapsed = bench.timed_loop(step, steps=4, warmup=2, pg=pg, local=local)
    q.put((rank, elapsed, len(calls)))
    pg.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_timed_loop_max_over_ranks_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    times = [t for _, t, _ in res]
    assert all(c == 6 for _, _, c in res)            # warmup 2 + steps 4 on every rank
    assert abs(times[0] - times[1]) < 1e-9           # every rank reports the same (max) time
    assert times[0] >= 4 * 0.03 * world * 0.95       # ... which is the slowest rank's


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
    # no GPU here: the binding is a no-op and leaves the affinity alone
    before = os.sched_getaffinity(0)
    assert bench.bind_to_gpu_numa_node(0) is None
    assert os.sched_getaffinity(0) == before
