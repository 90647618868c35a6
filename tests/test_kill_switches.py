"""The off path of every column-hint kill switch, against the oracle's full-size pin.

The single-GPU host path learns column classes from one proof and uses them for the next (prover.hip):
sparse columns skip their NTTs (ZK_SPARSE), narrow columns go up packed (ZK_NARROW), the AIR clock is derived instead
of uploaded (ZK_CLOCK), hinted sparse columns get no LDE in memory (ZK_VIRTUAL); the sharded host path has the same
hints (ZK_SHARD_HINTS).  (Round 6 folded ZK_LATENCY_SCHED and ZK_VM_PREFIX into their measured defaults: the upload
schedule is chosen per prover through zk_prover_set_upload_schedule, tested below with zk_prover_proof_info reporting
the schedule each proof ran.)  The switches are read once per process, so each off path runs in a child process: the
configs[2] trace (2^20, the c2_cipher_2p20 pin) proved three times from the host trace -- the first proof unhinted,
the later ones with whatever the switch leaves on -- must give the pinned proof every time, and the upload record must
show the switched-off class absent.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
pytestmark = pytest.mark.gpu

CHILD = r'''
import hashlib, json, sys
sys.path[:0] = [{root!r}, {pkg!r}, {tests!r}]
from golden_large import LARGE_CASES, large_inputs
from zkvm_amd.prover import GpuProver
c = next(c for c in LARGE_CASES if c["name"] == "c2_cipher_2p20")
ht, trace, pub, opts = large_inputs(c)
n = trace.shape[1]
out = {{"want": c["proof_sha256"], "single": [], "uploads": []}}
g = GpuProver(0, max_trace_len=n)
for _ in range(3):
    out["single"].append(hashlib.sha256(g.prove_host(trace, pub, opts)[0]).hexdigest())
    out["uploads"].append(g.upload_stats())
g.close()
if {sharded!r}:
    from zkvm_amd.sharded import ShardedProver
    sp = ShardedProver.loopback(2, 0, n)
    out["sharded"] = [hashlib.sha256(sp.prove(trace, pub, opts)[0]).hexdigest() for _ in range(3)]
    sp.close()
ht.close()
print("RESULT " + json.dumps(out), flush=True)
'''

SWITCHES = ["ZK_SPARSE", "ZK_NARROW", "ZK_CLOCK", "ZK_VIRTUAL", "ZK_SHARD_HINTS"]


@pytest.mark.parametrize("switch", SWITCHES)
def test_kill_switch_off_path_matches_pin(switch, tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD.format(root=str(ROOT), pkg=str(ROOT / "encrypt-zkvm_amd"), tests=str(ROOT / "tests"),
                                   sharded=switch == "ZK_SHARD_HINTS"))
    env = dict(os.environ, **{switch: "0"})
    r = subprocess.run([sys.executable, "-u", str(script)], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads(next(ln for ln in r.stdout.splitlines() if ln.startswith("RESULT "))[7:])
    assert out["single"] == [out["want"]] * 3
    hinted = out["uploads"][-1]  # the third proof: hints learned by the first two
    if switch == "ZK_SPARSE":
        assert hinted["sparse"] == []
    elif switch == "ZK_NARROW":
        assert hinted["narrow8"] == [] and hinted["narrow32"] == [] and hinted["sparse"]
    elif switch == "ZK_CLOCK":
        assert hinted["derived"] == [] and hinted["sparse"]
    elif switch == "ZK_SHARD_HINTS":
        assert out["sharded"] == [out["want"]] * 3


VM_CHILD = r'''
import hashlib, json, sys
sys.path[:0] = [{root!r}, {pkg!r}, {tests!r}]
from golden_large import LARGE_CASES
from zkvm_amd.prover import GpuProver, Program, ProofOptions
from zkvm_amd.workloads import make_workload, ops_for_trace_len
c = next(c for c in LARGE_CASES if c["name"] == "c2_cipher_2p20")
src = ops_for_trace_len(c["log_n"], c["generator"])
w = make_workload(src, seed=c["seed"])
prog = Program(src)
g = GpuProver(0, max_trace_len=prog.trace_len)
inputs = Program.encode_inputs(w.public, w.secret, w.server_key)
got = [hashlib.sha256(prog.prove_device(g, inputs, w.last_row, ProofOptions())[2]).hexdigest() for _ in range(3)]
g.close()
prog.close()
print("RESULT " + json.dumps({{"want": c["proof_sha256"], "got": got}}), flush=True)
'''


def test_vm_prove_prefix_matches_pin(tmp_path):
    """zk_vm_prove queues the preprocessed columns' commitment work ahead of the host stack pass (round 6: always; its
    ZK_VM_PREFIX switch was folded into the default after the A/B of profiles/r05k_vm_latency_ab_prefix.txt); the
    calls give configs[2]'s pinned proof, call after call (the first call builds the columns)."""
    script = tmp_path / "vm_child.py"
    script.write_text(VM_CHILD.format(root=str(ROOT), pkg=str(ROOT / "encrypt-zkvm_amd"), tests=str(ROOT / "tests")))
    r = subprocess.run([sys.executable, "-u", str(script)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads(next(ln for ln in r.stdout.splitlines() if ln.startswith("RESULT "))[7:])
    assert out["got"] == [out["want"]] * 3


SCHED_CHILD = r'''
import hashlib, json, sys, threading, time
sys.path[:0] = [{root!r}, {pkg!r}, {tests!r}]
from golden_large import LARGE_CASES, large_inputs
from zkvm_amd.prover import GpuProver
c = next(c for c in LARGE_CASES if c["name"] == "c2_cipher_2p20")
ht, trace, pub, opts = large_inputs(c)
n = trace.shape[1]
out = {{"want": c["proof_sha256"], "forced": {{}}}}
g = GpuProver(0, max_trace_len=n)
h = GpuProver(0, max_trace_len=n)
for sched in ("throughput", "latency"):
    g.set_upload_schedule(sched)
    got = []
    for _ in range(3):
        pr = g.prove_host(trace, pub, opts)[0]
        got.append((hashlib.sha256(pr).hexdigest(), g.proof_info()["schedule"], g.upload_stats()))
    out["forced"][sched] = got
g.set_upload_schedule("auto")
g.prove_host(trace, pub, opts)
out["auto_alone"] = g.proof_info()["schedule"]
# AUTO beside another proof: h proves in a loop on another thread; g starts while h is in flight
stop = threading.Event()
def busy():
    while not stop.is_set():
        h.prove_host(trace, pub, opts)
t = threading.Thread(target=busy)
t.start()
time.sleep(0.2)
out["auto_beside"], out["auto_beside_sha"] = [], []
for _ in range(3):
    pr = g.prove_host(trace, pub, opts)[0]
    out["auto_beside"].append(g.proof_info()["schedule"])
    out["auto_beside_sha"].append(hashlib.sha256(pr).hexdigest())
stop.set()
t.join()
out["info"] = g.proof_info()
g.close()
h.close()
ht.close()
print("RESULT " + json.dumps(out), flush=True)
'''


def test_upload_schedule_reported_and_pinned(tmp_path):
    """Each upload schedule, forced per prover (zk_prover_set_upload_schedule), is the one zk_prover_proof_info reports,
    and gives the pinned configs[2] proof with the hints in use (sparse, packed narrow and derived clock columns after
    the first proof); AUTO runs the latency schedule for a proof alone on the device and the throughput one for a proof
    that starts while another prover's proof is in flight (the C-ABI contract in include/zkvm_gpu.h)."""
    script = tmp_path / "sched_child.py"
    script.write_text(SCHED_CHILD.format(root=str(ROOT), pkg=str(ROOT / "encrypt-zkvm_amd"), tests=str(ROOT / "tests")))
    r = subprocess.run([sys.executable, "-u", str(script)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads(next(ln for ln in r.stdout.splitlines() if ln.startswith("RESULT "))[7:])
    for sched, got in out["forced"].items():
        assert [x[0] for x in got] == [out["want"]] * 3, sched
        assert [x[1] for x in got] == [sched] * 3, sched
        hinted = got[-1][2]
        assert hinted["sparse"] and hinted["narrow8"] and hinted["derived"], sched
    assert out["auto_alone"] == "latency"
    # (h's proofs run back to back: a call of g may start in the microseconds between two of them)
    assert out["auto_beside"].count("throughput") >= 2, out["auto_beside"]
    assert out["auto_beside_sha"] == [out["want"]] * 3
    assert out["info"]["hint_redos"] == 0 and out["info"]["hint_sets"] == 1
