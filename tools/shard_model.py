"""Measured decomposition and schedule model of the coset-sharded prover's per-rank time.

Two measurements of one 2^log_n proof, every rank of a G-way loopback proof on ONE GPU:
 (1) the R / S fit of earlier rounds: T_loop(G) = G R + S (+ in-process exchange copies), R the work every rank
     repeats, S the work divided among them; from G = 2, 4, 8 by least squares, per proof stage too (stage_split);
 (2) (round 6) the schedule model.  In the serialised measurement mode (zk_comm_set_measure) every rank's kernels and
     the exchange copies run on one stream in program order, and the library logs its schedule
     (zk_prover_shard_schedule): the compute segment between two exchange events (an exchange started, or the compute
     stream waiting for one), each segment's measured time (all G ranks' compute, serialised: the per-rank time is
     1/G of it; a segment that only the lead rank runs -- FRI layers >= 1, queries -- counts whole), and every
     exchange's bytes.  simulate() replays that exact dependency order for one rank on its own GPU: compute segments
     on the compute stream, each exchange on the exchange stream (FIFO) from the moment it is started, at the link
     model below, and a wait holds the compute stream until that exchange is done.  Overlap is what the code issues,
     not an assumption; `no_overlap` replays the same schedule with every exchange blocking.
Link model (unchanged since round 3, never measured on xGMI here): per-direction 76.8 GB/s per link, 70 % collective
efficiency, G - 1 links, 50 us per collective; a rank receives `bytes` per collective.  Not modelled: host gaps inside
segments are divided by G like the compute (tens of us each), and RCCL's kernels are assumed not to slow the compute
they overlap.
    python3 tools/shard_model.py [log_n] [steps]              (GPU box: both measurements, one JSON object)
    python3 tools/shard_model.py --schedule [log_n]            (GPU box: the schedule model only)
    python3 tools/shard_model.py --from profiles/<run>.json    (re-derive the stage split / projection, no GPU)
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


LINK_BPS = 76.8e9 * 0.7  # per-direction xGMI per link x collective efficiency
LAT_MS = 0.05


def xchg_ms(bytes_received, G):
    return LAT_MS + 1e3 * bytes_received / ((G - 1) * LINK_BPS)


def simulate(sched, G, overlap=True):
    """One rank's time for the logged schedule on G GPUs (see the module docstring).  Returns
    (total_ms, compute_ms, exchange_ms, exposed_ms, lead_ms)."""
    t = cq = comp = xtot = exposed = lead = 0.0
    done = {}
    for e in sched["entries"]:
        if "seg_ms" in e:
            d = e["seg_ms"] if e["lead"] else e["seg_ms"] / G
            t += d
            comp += d
            lead += d if e["lead"] else 0.0
        elif "start" in e:
            d = xchg_ms(e["bytes"], G)
            xtot += d
            if overlap:
                cq = max(t, cq) + d
                done[e["start"]] = cq
            else:
                exposed += d
                t += d
                done[e["start"]] = t
        elif "wait" in e:
            end = done[e["wait"]]
            if end > t:
                if overlap:
                    exposed += end - t
                t = end
    return t, comp, xtot, exposed, lead


def schedule_model(log_n, steps=3):
    """Loopback proofs at G = 2, 4, 8 in the measurement mode: schedules, and their replay (simulate)."""
    from zkvm_amd.prover import HostTrace, Program, ProofOptions, make_pub_inputs, vm_trace
    from zkvm_amd.sharded import ShardedProver
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    src = ops_for_trace_len(log_n, "cipher")
    w = make_workload(src, seed=1000)
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    n = trace.shape[1]
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    host = HostTrace(n)
    host.array[...] = trace
    prog = Program(src)
    inp = Program.encode_inputs(w.public, w.secret, w.server_key)
    out = {"log_n": log_n, "schedules": {}, "projection": {}, "link_model": {"per_link_gbs": LINK_BPS / 1e9,
                                                                            "latency_ms": LAT_MS, "links": "G - 1"}}
    proofs = set()
    for G in (2, 4, 8):
        sp = ShardedProver.loopback(G, max_trace_len=n)
        try:
            sp.set_measure(True)
            runs = {}
            sp.upload_trace(trace)
            for kind, fn in (("device", lambda: sp.prove(None, pub, ProofOptions(), n=n)[0]),
                             ("host", lambda: sp.prove(host.array, pub, ProofOptions())[0]),
                             ("vm", lambda: sp.prove_program(prog, inp, w.last_row)[2])):
                best = None
                for _ in range(steps + 1):  # the first proof of each kind builds tables: dropped
                    proofs.add(fn())
                    sc = sp.schedule()
                    tot = sum(e.get("seg_ms", 0.0) for e in sc["entries"])
                    if best is None or tot < best[0]:
                        best = (tot, sc)
                runs[kind] = best[1]
                print(f"G={G} {kind}: {best[0]:.2f} ms of serialised compute", file=sys.stderr, flush=True)
            sp.set_measure(False)
        finally:
            sp.close()
        out["schedules"][G] = runs
    host.close()
    prog.close()
    assert len(proofs) == 1, "loopback world sizes / trace sources disagree on the proof bytes"
    out["projection"] = project(out["schedules"])
    return out


def split_sweep(log_n, reps=(0, 2, 4, 6, 8, 12, 16, 28), steps=2):
    """The replicated-column count of the trace interpolation (zk_comm_set_trace_split) swept per world size: the
    device-trace and vm schedules in the measurement mode, replayed per rank (the library's default table comes from
    this)."""
    from zkvm_amd.prover import Program, ProofOptions, make_pub_inputs, vm_trace
    from zkvm_amd.sharded import ShardedProver
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    src = ops_for_trace_len(log_n, "cipher")
    w = make_workload(src, seed=1000)
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    n = trace.shape[1]
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    prog = Program(src)
    inp = Program.encode_inputs(w.public, w.secret, w.server_key)
    out = {"log_n": log_n, "sweep": {}}
    proofs = set()
    for G in (2, 4, 8):
        sp = ShardedProver.loopback(G, max_trace_len=n)
        res = {}
        try:
            sp.set_measure(True)
            for kind in ("device", "vm"):
                for rep in reps:
                    if kind == "vm" and rep > 12:
                        continue
                    sp.set_trace_split(rep)
                    best = None
                    for _ in range(steps + 1):
                        if kind == "device":
                            sp.upload_trace(trace)
                            proofs.add(sp.prove(None, pub, ProofOptions(), n=n)[0])
                        else:
                            proofs.add(sp.prove_program(prog, inp, w.last_row)[2])
                        sc = sp.schedule()
                        tot = sum(e.get("seg_ms", 0.0) for e in sc["entries"])
                        if best is None or tot < best[0]:
                            best = (tot, sc)
                    t, comp, x, exp_, lead = simulate(best[1], G)
                    res.setdefault(kind, {})[rep] = {"per_rank_ms": round(t, 2), "compute_ms": round(comp, 2),
                                                     "exchange_ms": round(x, 2), "exposed_ms": round(exp_, 2)}
                    print(f"G={G} {kind} rep={rep}: {t:.2f} ms per rank (compute {comp:.2f}, exposed {exp_:.2f})",
                          file=sys.stderr, flush=True)
            sp.set_trace_split(-1)
        finally:
            sp.close()
        out["sweep"][G] = res
    prog.close()
    assert len(proofs) == 1, "the split changed the proof bytes"
    return out


def project(schedules):
    """Per trace source and G: the replayed per-rank time with the code's overlap and with every exchange blocking, and
    the R / S fit of the serialised compute (sum of segments at G = G R + S)."""
    res = {}
    kinds = sorted(set().union(*[set(v) for v in schedules.values()]))
    for kind in kinds:
        rec = {}
        tot = {}
        for G, runs in schedules.items():
            if kind not in runs:
                continue
            G = int(G)
            sc = runs[kind]
            t, comp, x, exp_, lead = simulate(sc, G)
            tn = simulate(sc, G, overlap=False)[0]
            rec[G] = {"per_rank_ms": round(t, 2), "no_overlap_ms": round(tn, 2), "compute_ms": round(comp, 2),
                      "exchange_ms": round(x, 2), "exposed_exchange_ms": round(exp_, 2), "lead_only_ms": round(lead, 2),
                      "collectives": sum(1 for e in sc["entries"] if "start" in e),
                      "received_mb": round(sum(e["bytes"] for e in sc["entries"] if "start" in e) / 1e6, 1)}
            tot[G] = sum(e["seg_ms"] for e in sc["entries"] if "seg_ms" in e and not e["lead"])
        if len(tot) >= 2:
            Gs = np.array(sorted(tot), dtype=float)
            A = np.stack([Gs, np.ones(len(Gs))], axis=1)
            (R, S), *_ = np.linalg.lstsq(A, np.array([tot[int(g)] for g in Gs]), rcond=None)
            rec["fit_all_rank_segments"] = {"replicated_ms_R": round(float(R), 3), "divided_ms_S": round(float(S), 3)}
        res[kind] = rec
    return res


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--from":
        res = json.loads(Path(sys.argv[2]).read_text())
        out = {"source": sys.argv[2]}
        if "schedules" in res:
            out["projection"] = project(res["schedules"])
        if any(k in res for k in ("stage_ms", "stage_ms_host", "stage_ms_vm")):
            out["stage_split"] = stage_split(res)
        print(json.dumps(out, indent=1))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "--sweep":
        log_n = int(sys.argv[2]) if len(sys.argv) > 2 else 22
        print(json.dumps(split_sweep(log_n)))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "--schedule":
        log_n = int(sys.argv[2]) if len(sys.argv) > 2 else 22
        print(json.dumps(schedule_model(log_n)))
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
