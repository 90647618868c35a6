"""Measured decomposition of the coset-sharded prover's per-rank time.

Loopback ranks run every rank of a G-way sharded proof on ONE GPU, so the wall time of a loopback proof is
    T_loop(G) = G * R + S + X(G)
with R the work every rank repeats (interpolation, DEEP coefficients, FRI layers >= 1, host steps), S the work that
is divided among the ranks (LDEs, evaluation, hashing, layer 0) and X the in-process exchange copies (device-local,
small).  From G = 2, 4, 8 this fits R and S (least squares); the per-rank time on G separate GPUs is then
R + S / G + exchange(G), the exchange priced from the bytes rank 0 received in the loopback proof at an assumed xGMI
rate ("projection").
The same fit per proof stage (stage_split: the stage marks of the loopback proofs, each stage's time summed over the
G ranks the process drives) says where R and S sit.
    python3 tools/shard_model.py [log_n] [steps]      (GPU box; prints one JSON object)
    python3 tools/shard_model.py --from profiles/<run>.json   (the per-stage split of a committed run, no GPU)
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "encrypt-zkvm_amd"))


def stage_split(res):
    """Per stage s: T_s(G) = G R_s + S_s over G = 2, 4, 8 (least squares) for each stage-time record of the run."""
    Gs = np.array([2.0, 4.0, 8.0])
    A = np.stack([Gs, np.ones(3)], axis=1)
    out = {}
    for key in ("stage_ms", "stage_ms_host", "stage_ms_vm"):
        if key not in res:
            continue
        rec = {str(g): v for g, v in res[key].items()}
        stages = sorted(set().union(*[set(rec[str(g)]) for g in (2, 4, 8)]), key=lambda k: -rec["2"].get(k, 0))
        split = {}
        for st in stages:
            T = np.array([rec[str(g)].get(st, 0.0) for g in (2, 4, 8)])
            (R, S), *_ = np.linalg.lstsq(A, T, rcond=None)
            split[st] = {"R_ms": round(float(R), 3), "S_ms": round(float(S), 3), "per_rank_g8_ms": round(float(R + S / 8), 3)}
        split["total"] = {k: round(sum(v[k] for v in split.values()), 3) for k in ("R_ms", "S_ms", "per_rank_g8_ms")}
        out[key] = split
    return out


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--from":
        res = json.loads(Path(sys.argv[2]).read_text())
        print(json.dumps({"source": sys.argv[2], "stage_split": stage_split(res)}, indent=1))
        return
    from zkvm_amd.prover import HostTrace, Program, ProofOptions, make_pub_inputs, vm_trace
    from zkvm_amd.sharded import ShardedProver
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    src = ops_for_trace_len(log_n, "cipher")
    w = make_workload(src, seed=1000)
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    n = trace.shape[1]
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    host = HostTrace(n)  # page-locked copy: the host-resident call shape (each rank uploads its column slice)
    host.array[...] = trace
    prog = Program(src)
    inp = Program.encode_inputs(w.public, w.secret, w.server_key)
    res = {"log_n": log_n, "steps": steps, "loopback_ms": {}, "loopback_host_ms": {}, "loopback_vm_ms": {},
           "stage_ms": {}, "stage_ms_vm": {}}
    proofs = set()

    def timed(sp, fn):
        for _ in range(2):
            proofs.add(fn())
        t0 = time.perf_counter()
        for _ in range(steps):
            proofs.add(fn())
        return 1e3 * (time.perf_counter() - t0) / steps

    for G in (2, 4, 8):
        sp = ShardedProver.loopback(G, max_trace_len=n)
        try:
            res["loopback_host_ms"][G] = timed(sp, lambda: sp.prove(host.array, pub, ProofOptions())[0])
            res.setdefault("received", {}).setdefault("host", {})[G] = sp.exchange_stats()
            res.setdefault("stage_ms_host", {})[G] = {k: round(v, 3) for k, v in sp.stage_times().items()}
            sp.upload_trace(trace)
            res["loopback_ms"][G] = timed(sp, lambda: sp.prove(None, pub, ProofOptions(), n=n)[0])
            res["received"].setdefault("device", {})[G] = sp.exchange_stats()
            res["stage_ms"][G] = {k: round(v, 3) for k, v in sp.stage_times().items()}
            # vm::prove sharded: every loopback rank also writes its own trace (zk_vm_prove_sharded), so the VM's
            # host stack pass and row kernels are counted once per rank, like the replicated work they are
            res["loopback_vm_ms"][G] = timed(sp, lambda: sp.prove_program(prog, inp, w.last_row)[2])
            res["stage_ms_vm"][G] = {k: round(v, 3) for k, v in sp.stage_times().items()}
        finally:
            sp.close()
        print(f"G={G}: {res['loopback_ms'][G]:.2f} ms per loopback proof (device trace), "
              f"{res['loopback_host_ms'][G]:.2f} (host trace), {res['loopback_vm_ms'][G]:.2f} (vm_prove)",
              file=sys.stderr, flush=True)
    host.close()
    prog.close()
    assert len(proofs) == 1, "loopback world sizes disagree on the proof bytes"
    Gs = np.array([2.0, 4.0, 8.0])
    A = np.stack([Gs, np.ones(3)], axis=1)
    for key, name in (("loopback_ms", "fit"), ("loopback_host_ms", "fit_host"), ("loopback_vm_ms", "fit_vm")):
        T = np.array([res[key][g] for g in (2, 4, 8)])
        (R, S), *_ = np.linalg.lstsq(A, T, rcond=None)
        res[name] = {"replicated_ms_R": round(float(R), 3), "divided_ms_S": round(float(S), 3),
                     "residuals_ms": [round(float(x), 3) for x in (T - A @ np.array([R, S]))]}
    # Per rank on G separate GPUs: R + S / G + the exchanges, priced from the bytes rank 0 received in the loopback
    # proof (the same collectives and volumes an RCCL rank sees) at the link model of DESIGN.md section 7: per-direction
    # xGMI 76.8 GB/s per link, 70 % collective efficiency, G - 1 links, 50 us per collective, no overlap with compute
    link = 76.8e9 * 0.7
    res["projection"] = {}
    for kind, fit in (("device", "fit"), ("host", "fit_host")):
        R, S = res[fit]["replicated_ms_R"], res[fit]["divided_ms_S"]
        proj = {}
        for G in (2, 4, 8):
            st = res["received"][kind][G]
            nbytes = sum(v[1] for v in st.values())
            calls = sum(v[2] for v in st.values())
            x_ms = 1e3 * nbytes / ((G - 1) * link) + 0.05 * calls
            proj[G] = {"per_rank_ms": round(R + S / G + x_ms, 2), "exchange_ms": round(x_ms, 2),
                       "received_mb": round(nbytes / 1e6, 1), "collectives": calls}
        res["projection"][kind] = proj
    res["received"] = {k: {G: {c: [round(v[1] / 1e6, 2), v[2]] for c, v in d.items()} for G, d in m.items()}
                       for k, m in res["received"].items()}
    res["stage_split"] = stage_split(res)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
