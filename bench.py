"""Benchmark: STARK prove throughput (trace-steps/s) on MI355X, BASELINE.json metric.

Workload (BASELINE.json configs[2]): a 2^20-step Encrypt-zkVM program mixing READ2/ADD2/SMUL
ciphertext ops (zkvm_amd.workloads.cipher_mix_program), proved with the reference options
ProofOptions(32, 8, 0, None, 8, 127) (vm/src/lib.rs:20).  One step = one full Prover::prove of that
trace: trace LDE + commitment, constraint evaluation, composition commitment, OOD/DEEP, FRI,
queries and proof bytes.  The trace is generated once on the host (VM, untimed) straight into page-locked host memory; each timed step
is one zk_prove call from that host-resident trace to proof bytes (the reference's call shape: vm/src/lib.rs
builds a TraceTable in host memory and hands it to Prover::prove).  The library uploads it in column groups
on a copy stream, overlapped with the interpolation and, with two provers in flight, with the other proof's
kernels.  Beside `value` the line reports device_resident_ms (the trace already in HBM), pageable_host_ms
(the trace in ordinary pageable memory), latency_ms (one prove() call alone on the GPU) and steady_state_ms (the
host-resident proofs over a 100-proof window).  The default window is 60 proofs: a 20-proof window pays the run's two
ends -- nothing to compute before the first column group is up, fewer co-runners for the last proofs -- about 1 %
on the round-5 path (11.11 / 11.17 ms per proof against 11.06 / 11.04 at 60 and 11.02 / 11.05 at 100, one box;
tools/inflight_timeline.py), and 60 proofs are 0.7 s of GPU time.

Proofs in flight (--inflight P, default 3): each GPU holds P independent provers (own HBM buffers and
compute streams, zk_prover objects; one upload stream per device) driven by P host threads, so one prover's trace
upload, host-side transcript round trips and proof tail overlap the others' kernels.  P + 1 streams fit HIP's
default 4 hardware queues at P = 3 (A/B at 4 queues, three passes: 11.53-11.56 ms per proof at P = 3, 11.52-11.58
at P = 2, 11.75-11.79 at P = 4; profiles/r04_ab_queues.txt; final round-4 tree: 11.30-11.37 at P = 3 against
11.41-12.32 at P = 2 and 11.65-11.68 at P = 4, profiles/r04v_ab_inflight.txt), so the line needs no GPU_MAX_HW_QUEUES setting
(queues_ab re-runs it at 16).  The K timed steps are K complete proofs, dealt round-robin to the provers;
per-proof latency is stage_ms.

Multi-GPU (one process per GPU, torchrun): every rank proves its own independent trace (weak
scaling, no data-path collective); the driver's barrier + max-over-ranks timing gives the
whole-job rate.  rank 0 prints one JSON line.  Each process pins its host threads to the NUMA node of its
GPU (bind_to_gpu_numa_node; ZK_NUMA_BIND=0 turns it off), so its page-locked trace lives behind its own PCIe root.

--config5 (BASELINE.json configs[4]): the same workload at 128-bit conjectured security,
ProofOptions(43, 8, 0, Quadratic, 8, 127): composition, OOD, DEEP and FRI over the quadratic extension.

--sharded (BASELINE.json configs[3], e.g. --log-n 22): ONE proof per step with the LDE domain sharded
by coset over all ranks (zk_prove_sharded, RCCL over xGMI: all-to-all of leaf digests and composition
coefficient slices, all-gathers of subtree roots, FRI layer 1 and openings); strong scaling.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
for p in (ROOT, ROOT / "encrypt-zkvm_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (/opt/skills/guides/MI355X_MICROARCH.md)
# f128 operation throughput of this build's field arithmetic, whole chip, measured by
# tools/ubench/mul_ubench.hip (profiles/r01_ubench_field_ops.txt): the VALU ceiling of the NTT
FE_MUL_PEAK = 536.78e9
FE_ADD_PEAK = 2922.68e9
FE_SUB_PEAK = 3251.22e9
STEADY_PROOFS = 100  # steady_state_ms window (host-resident, same provers; outside the headline)
METRIC = "STARK prove: trace-steps/sec at 2^20 steps; achieved HBM GB/s vs 8 TB/s peak"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ZK_BENCH_REHEARSE=1: rehearse the multi-GPU flow on fewer GPUs than ranks (several ranks per GPU): ranks share GPUs
# round robin and the sharded leg exchanges through zk_comm_create_host over the TCP host group instead of RCCL (which
# refuses two ranks on one device).  Same code path otherwise (barriers, max over ranks, rank 0's line, the sharded sub-record).
REHEARSE = os.environ.get("ZK_BENCH_REHEARSE", "0") == "1"


def setup_dist(n_gpus):
    """One process per GPU, torch-free: the library's own HIP runtime and RCCL (native.runtime_info(), recorded in the
    line) and a TCP host group for barriers, max over ranks and the RCCL id (zkvm_amd.hostgroup; torchrun's
    environment).  torch is never imported -- it bundles another libamdhip64 / librccl (ROCm 7.0), and the library
    would run on whichever copy came first.  --torch-runtime imports it first on purpose (the runtime A/B)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    from zkvm_amd import native
    native.lib()  # fail loudly without the HIP library
    ndev = native.device_count()
    if REHEARSE:
        local %= max(1, ndev)
    pg = None
    if world > 1:
        from zkvm_amd.hostgroup import HostGroup
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        pg = HostGroup.from_env()
    if ndev > 0 and os.environ.get("ZK_NUMA_BIND", "1") != "0":
        HOST["numa_node"] = bind_to_gpu_numa_node(local)
        if world > 1:
            log(f"[rank {rank}] GPU {local}: host threads on NUMA node {HOST['numa_node']}")
    return world, rank, local, pg


HOST = {"numa_node": None}  # the NUMA node this process's host threads were pinned to (bind_to_gpu_numa_node)


def _cpulist(text):
    cpus = set()
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def bind_to_gpu_numa_node(local):
    """Pin this rank's host threads to the NUMA node its GPU hangs off (with several GPUs per host): the page-locked
    trace is then allocated and written on that node, and each upload reads memory behind its own PCIe root rather
    than across the socket link.  Threads started later (the VM's) inherit it.  The device's PCI address comes from
    the library's runtime (zk_device_pci_bus_id).  Returns the node, or None where the topology is not exposed
    (nothing changes then)."""
    try:
        from zkvm_amd import native
        bdf = native.pci_bus_id(local).lower()
        node = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
        if node < 0:
            return None
        cpus = _cpulist(open(f"/sys/devices/system/node/node{node}/cpulist").read()) & os.sched_getaffinity(0)
        if not cpus:
            return None
        os.sched_setaffinity(0, cpus)
        return node
    except Exception:
        return None


def _sync(local):
    from zkvm_amd import native
    if native.device_count() > 0:
        native.synchronize(local)


def barrier(pg, local):
    """Device sync, host barrier over every rank, device sync (the timed region's brackets)."""
    _sync(local)
    if pg is not None:
        pg.barrier()
        _sync(local)


def max_over_ranks(pg, value, local):
    return value if pg is None else pg.max(value)


def timed_loop(step, steps: int, warmup: int, pg, local: int) -> float:
    """W untimed warmup steps, then exactly K steps bracketed by barrier + device sync on both
    sides; returns the max over ranks of the elapsed wall time (seconds)."""
    for _ in range(warmup):
        step()
    barrier(pg, local)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    barrier(pg, local)
    return max_over_ranks(pg, time.perf_counter() - t0, local)


def run_proofs(fns, count: int):
    """count proofs dealt round-robin to the provers' step functions, one host thread per prover
    (the library call releases the GIL; a prover object is used by one thread at a time)."""
    P = len(fns)
    share = [count // P + (1 if k < count % P else 0) for k in range(P)]
    if P == 1:
        for _ in range(share[0]):
            fns[0]()
        return
    errs = []

    def run(k):
        try:
            for _ in range(share[k]):
                fns[k]()
        except BaseException as e:  # re-raised in the caller
            errs.append(e)

    ths = [threading.Thread(target=run, args=(k,)) for k in range(P) if share[k]]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errs:
        raise errs[0]


def cpu_baseline(log_n: int, config5: bool = False, all_cores: int = 0, repeats: int = 3):
    """The oracle's single-threaded CPU prove (the build's restatement of the reference path; the
    reference Rust prover cannot be built here) on a bounded sample of the same generator."""
    from oracle import oracle as orc
    from zkvm_amd.prover import vm_trace
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    orc.build()
    src = ops_for_trace_len(log_n, "cipher")
    w = make_workload(src, seed=77)
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    pub = orc.make_pub(h, outputs)
    opts = orc.default_options(num_queries=43, field_extension=2) if config5 else orc.default_options()
    runs = []
    for k in range(max(1, repeats)):  # each CPU config timed 3x in the same invocation, median
        log(f"cpu baseline: 2^{log_n} sample, proof {k + 1} of {repeats} ...")
        t0 = time.perf_counter()
        orc.prove(trace, pub, opts)
        runs.append(time.perf_counter() - t0)
    dt = sorted(runs)[len(runs) // 2]
    n = trace.shape[1]
    out = {"value": n / dt, "unit": "trace-steps/s", "cores": 1, "kind": "port",
           "runs_s": [round(r, 2) for r in runs],
           "sample": f"oracle or_prove (C, 1 thread), median of {len(runs)} proofs of one 2^{log_n}-step trace of the "
                     f"same cipher-mix generator, {'config-5' if config5 else 'reference'} options: {dt:.1f} s; a "
                     f"2^{log_n} sample of the 2^20 config (the CPU prover's time per step grows with log n: on a "
                     f"GPU box's host one proof of configs[2]'s own 2^20 trace took 95.8 s, 10.9 k trace-steps/s, "
                     f"profiles/r04n_cpu_baseline_2p20.json), so this figure flatters the CPU by ~10-20 %"}
    if all_cores > 1:
        # the reference prover is single-threaded (no rayon), so its whole-host throughput is one proof per
        # core: all_cores threads each prove the same trace at once (ctypes releases the GIL; the oracle
        # keeps no global state)
        errs = []

        def one():
            try:
                orc.prove(trace, pub, opts)
            except BaseException as e:  # re-raised below
                errs.append(e)

        ths = [threading.Thread(target=one) for _ in range(all_cores)]
        log(f"cpu baseline: {all_cores} concurrent 2^{log_n} proofs ...")
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        dta = time.perf_counter() - t0
        if errs:
            raise errs[0]
        out["all_cores"] = {"value": all_cores * n / dta, "unit": "trace-steps/s", "cores": all_cores,
                            "sample": f"{all_cores} concurrent single-thread oracle proofs of the same 2^{log_n} "
                                      f"trace: {dta:.1f} s"}
    return out


def cpu_headline(trace, pub, opts, gpu_proof: bytes, log_n: int, runs: int = 3):
    """cpu_baseline.value: the median of `runs` proofs of the headline workload's own 2^log_n trace by the oracle's
    single-threaded or_prove (the build's C restatement of the reference prover, which cannot be built here), each on
    its own core of this host (each config 3x in the same invocation, median).  The runs go concurrently,
    one thread each (ctypes releases the GIL; the oracle keeps no global state), so the three cost one proof's wall
    time; every proof must equal the GPU's byte for byte."""
    import ctypes as C
    from oracle import oracle as orc
    orc.build()
    opub = orc.PubInputs()
    C.memmove(opub.program_hash, bytes(pub.program_hash), 32)
    C.memmove(opub.stack_outputs, bytes(pub.stack_outputs), 256)
    opub.lwe_size, opub.delta = pub.lwe_size, pub.delta
    oopts = orc.default_options(num_queries=opts.num_queries, field_extension=opts.field_extension)
    log(f"cpu baseline: {runs} concurrent single-thread oracle proofs of the 2^{log_n} workload trace ...")
    times, proofs, errs = [None] * runs, [None] * runs, []

    def one(k):
        try:
            t0 = time.perf_counter()
            proofs[k] = orc.prove(trace, opub, oopts)[0]
            times[k] = time.perf_counter() - t0
        except BaseException as e:  # re-raised below
            errs.append(e)

    ths = [threading.Thread(target=one, args=(k,)) for k in range(runs)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    wall = time.perf_counter() - t0
    if errs:
        raise errs[0]
    dt = sorted(times)[len(times) // 2]
    n = trace.shape[1]
    return {"value": n / dt, "unit": "trace-steps/s", "cores": 1, "kind": "port",
            "runs_s": [round(t, 2) for t in times], "median_s": round(dt, 2), "wall_s": round(wall, 2),
            "proof_equals_gpu_proof": all(p == gpu_proof for p in proofs),
            "sample": f"oracle or_prove (C, 1 thread per proof): median of {runs} proofs of the timed workload's own "
                      f"2^{log_n}-step trace (input set 0, the configs[2] pin's trace) with the same options, run "
                      f"concurrently on {runs} cores of this host ({dt:.1f} s median); the reference prover (winterfell "
                      f"0.9, single-threaded) cannot be built here"}


def host_cores(req: int) -> int:
    """Threads for the all-cores CPU sample: the requested count, else this process's CPU share (affinity,
    OMP_NUM_THREADS: the GPU box sets it to the box's share of a larger machine), capped at 16."""
    if req >= 0:
        return req
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, min(n, 16))


PINS = ROOT / "tests" / "golden" / "large" / "cases.json"


def find_pin(log_n: int, seed: int, opts, generator: str = "cipher"):
    """The committed full-size oracle pin (tests/golden/large, tools/gen_golden_large.py) of exactly this workload --
    trace length, generator, seed and proof options -- or None.  The bench's rank-0 replica workload (seed 1000,
    2^20) is configs[2]'s pin c2_cipher_2p20 (c4_cipher_2p20_quad with --config5), the sharded leg's is c3_cipher_2p22."""
    if not PINS.exists():
        return None
    want = {"num_queries": opts.num_queries, "blowup": opts.blowup_factor, "grinding": opts.grinding_factor,
            "field_extension": opts.field_extension, "fri_folding": opts.fri_folding_factor,
            "fri_rem_max_deg": opts.fri_remainder_max_degree}
    for c in json.loads(PINS.read_text())["cases"]:
        if c["log_n"] == log_n and c["seed"] == seed and c["generator"] == generator and c["options"] == want:
            return c
    return None


def pin_check(proof: bytes, pin):
    """{"pin": name, "proof_matches_pin": bool} (None without a pin)."""
    import hashlib
    if pin is None:
        return None
    return {"pin": pin["name"], "proof_matches_pin": len(proof) == pin["proof_len"] and
            hashlib.sha256(proof).hexdigest() == pin["proof_sha256"]}


def all_ranks_true(pg, ok: bool, local: int) -> bool:
    """True iff ok holds on every rank (a MAX over ranks of the failure flag)."""
    return max_over_ranks(pg, 0.0 if ok else 1.0, local) == 0.0


def pmc_traffic(kernel: str, config5: bool = False):
    """HBM traffic of the kernel from the committed rocprofv3 --pmc passes of the same configuration
    (tools/pmc_traffic.py, tools/gpu_profile.sh): per launch and per proof over the LAST (steady-state, hinted) proof
    of a one-prover run, the ratio to that proof's algorithmic bytes, and whether the profile was taken on the
    sources this bench runs (source hash, zkvm_amd.treehash)."""
    f = ROOT / "profiles" / ("pmc_traffic_config5.json" if config5 else "pmc_traffic.json")
    if not f.exists():
        return None
    try:
        from zkvm_amd.treehash import source_hash
        d = json.loads(f.read_text())
        return {"per_launch_bytes": d.get("per_launch_bytes", {}).get(kernel),
                "per_proof_bytes": d.get("per_proof_bytes", {}).get(kernel),
                "alg_per_proof_bytes": d.get("alg_per_proof_bytes", {}).get(kernel),
                "traffic_ratio": d.get("traffic_ratio", {}).get(kernel), "scope": d.get("scope"),
                "profile": f"profiles/{f.name}", "profile_tree": d.get("tree"),
                "profile_tree_matches": d.get("tree") == source_hash()}
    except Exception:
        return None


def run_proofs_timed(fns, count: int, pg, local: int) -> float:
    """count proofs over the provers' step functions, bracketed by barrier + device sync; max over ranks (s)."""
    barrier(pg, local)
    t0 = time.perf_counter()
    run_proofs(fns, count)
    barrier(pg, local)
    return max_over_ranks(pg, time.perf_counter() - t0, local)


def pmc_valu(kernel: str):
    """Hardware VALU issue of the kernel from the committed rocprofv3 SQ/GRBM pass (tools/pmc_valu.py):
    SQ_INSTS_VALU over the 1024 SIMDs' 2-cycle issue slots (a plain wave64 VALU instruction takes one) --
    the hardware roofline of an integer-VALU-bound kernel, independent of this build's own field ops."""
    f = ROOT / "profiles" / "pmc_valu.json"
    if not f.exists():
        return None
    try:
        from zkvm_amd.treehash import source_hash
        d = json.loads(f.read_text())
        k = d["kernels"].get(kernel)
    except Exception:
        return None
    if not k:
        return None
    return {"bound": "valu-issue", "slot_util": round(k["slot_util"], 3), "clock_ghz": round(k["clock_ghz"], 2),
            "valu_instr_per_launch": k["valu_instr"] / k["launches"], "peak": "1024 SIMDs x 1 wave64 VALU instr / 2 cycles",
            "source": "profiles/pmc_valu.json (rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE, tools/pmc_valu.py)",
            "profile_tree": d.get("tree"), "profile_tree_matches": d.get("tree") == source_hash()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed proofs before the timed region (default 3 per prover in flight; the first proof of "
                         "each prover builds its per-size tables)")
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--cpu-log-n", type=int, default=18)  # ~20 s of single-core oracle work (--cpu-sample)
    ap.add_argument("--cpu-sample", action="store_true",
                    help="also time the 2^cpu-log-n CPU sample (median of 3) and the all-cores figure")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-cores", type=int, default=-1,
                    help="threads of the all-cores CPU sample (-1: the host share, at most 16; 0: skip it)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--inflight", type=int, default=3, help="independent provers (proofs in flight) per GPU")
    ap.add_argument("--sharded", action="store_true", help="one proof sharded over all ranks (configs[3])")
    ap.add_argument("--sharded-log-n", type=int, default=22,
                    help="trace length of the sharded sub-record that runs when WORLD_SIZE > 1 (0: skip it)")
    ap.add_argument("--no-compare", action="store_true",
                    help="skip the device-resident / pageable / latency comparison legs (profiler passes)")
    ap.add_argument("--ab", action="store_true",
                    help="A/B runs: of the comparison legs keep only steady_state, device-resident and latency")
    ap.add_argument("--config5", action="store_true",
                    help="128-bit security options (configs[4]): 43 queries, FieldExtension::Quadratic")
    ap.add_argument("--input-sets", type=int, default=4,
                    help="input sets of the workload program the timed proofs rotate through (fresh secrets, public "
                         "inputs and random last rows; set 0 is the pinned seed-1000 workload)")
    ap.add_argument("--upload-schedule", choices=["auto", "throughput", "latency"], default="auto",
                    help="how the host trace goes up (zk_prover_set_upload_schedule) in the timed proofs; auto: the "
                         "latency schedule for a proof alone on the GPU, else the throughput one (profile passes with "
                         "--inflight 1 pass throughput, so their proofs are those of the default P = 3 line)")
    ap.add_argument("--torch-runtime", action="store_true",
                    help="import torch before the library (runtime A/B only): the library then runs on torch's bundled "
                         "HIP runtime and RCCL instead of the /opt/rocm copies it links")
    args = ap.parse_args()
    if args.torch_runtime:
        import torch  # noqa: F401  (maps torch/lib/libamdhip64.so first; the library shares it)
    # HIP's hardware queues per process: whatever the environment gives (the runtime's default is 4, which the GPU
    # boxes of this pool also export); reported in the line, and queues_ab re-runs the workload at the other setting
    if args.sharded:
        return run_sharded(args)

    world, rank, local, pg = setup_dist(args.gpus)
    from zkvm_amd import native
    from zkvm_amd.prover import GpuProver, HostTrace, Program, ProofOptions, make_pub_inputs
    from zkvm_amd.workloads import make_workload, ops_for_trace_len, padded_length, trace_length

    native.lib()  # fail loudly without the HIP library
    src = ops_for_trace_len(args.log_n, "cipher")
    program_ops = sum(1 for ln in src.splitlines() if ln.split("#")[0].strip())  # #program ops
    padded_ops = padded_length(src)
    w = make_workload(src, seed=1000 + rank)
    n = trace_length(src)
    # the VM writes its TraceTable straight into page-locked host memory (zk_host_alloc): the host-resident
    # trace the timed region starts from (vm/src/lib.rs:18 builds it, :26 hands it to prove)
    host = HostTrace(n)
    S = max(1, args.input_sets)
    # vm::prove's front half (vm/src/lib.rs:13-18) in the reference's two steps: Program::compile (parse, pad,
    # hash: the sequential Rescue sponge, once per program) and Processor::run + trace on this run's inputs
    # (a sequential stack pass plus threaded row writes), timed separately; neither is in the timed region
    t0 = time.perf_counter()
    prog = Program(src)
    t1 = time.perf_counter()
    trace, outputs = prog.trace(w.public, w.secret, w.server_key, w.last_row, out=host)
    t2 = time.perf_counter()
    h = prog.hash
    vm_rec = {"compile_ms": round(1e3 * (t1 - t0), 1), "trace_ms": round(1e3 * (t2 - t1), 1),
              "threads": os.environ.get("ZK_VM_THREADS") or os.environ.get("OMP_NUM_THREADS") or os.cpu_count()}
    log(f"[rank {rank}] VM: n={n} compile {vm_rec['compile_ms']} ms, trace {vm_rec['trace_ms']} ms")
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    # the other input sets of the same program: fresh secrets, public inputs and random last rows, each trace in its
    # own page-locked buffer (the timed proofs rotate through all S, as a server proving fresh inputs would)
    sets = [(trace, pub)]
    extra_hosts = []
    for k in range(1, S):
        wk = make_workload(src, seed=5000 + 16 * rank + k)
        hk = HostTrace(n)
        extra_hosts.append(hk)
        tk, ok = prog.trace(wk.public, wk.secret, wk.server_key, wk.last_row, out=hk)
        sets.append((tk, make_pub_inputs(h, ok, wk.server_key.lwe_size(), wk.server_key.parameters.delta)))
    opts = ProofOptions(43, 8, 0, 2, 8, 127) if args.config5 else ProofOptions()
    min_sec = 128 if args.config5 else 95
    opts_str = "ProofOptions(43, 8, 0, Quadratic, 8, 127)" if args.config5 else "ProofOptions(32, 8, 0, None, 8, 127)"
    P = max(1, args.inflight)
    provers = [GpuProver(local, max_trace_len=n, max_blowup=opts.blowup_factor) for _ in range(P)]
    for g_ in provers:
        g_.set_upload_schedule(args.upload_schedule)
    # the schedule the timed proofs ran (auto: three provers in flight keep each other company)
    timed_sched = args.upload_schedule if args.upload_schedule != "auto" else ("throughput" if P > 1 else "latency")
    gpu = provers[0]
    last = [None] * P

    def host_step(k, tr):
        def f():
            last[k] = provers[k].prove_host(tr, pub, opts)[0]
        return f

    # proofs per input set: every proof of a set must be the same bytes, whichever prover made it
    set_proofs = [None] * S
    nxt = [0]
    lock = threading.Lock()

    def rotating_step(k):
        def f():
            with lock:
                i = nxt[0] % S
                nxt[0] += 1
            tr, pb = sets[i]
            pr = provers[k].prove_host(tr, pb, opts)[0]
            with lock:
                if set_proofs[i] is None:
                    set_proofs[i] = pr
                elif set_proofs[i] != pr:
                    raise AssertionError(f"input set {i}: two proofs of the same trace differ")
            if i == 0:
                last[k] = pr
        return f

    # ---- value: zk_prove from the host-resident (page-locked) traces to proof bytes, P proofs in flight, rotating
    # through the S input sets
    fns = [rotating_step(k) for k in range(P)]
    # warm-up: exactly --warmup untimed proofs, dealt round-robin (each prover's first proof builds its per-size
    # tables; the next ones pay page faults and clock ramp-up: 18.9, 14.5, 14.2, then 13.9 ms,
    # tools/proof_times.py); the default is three per prover
    warm = args.warmup if args.warmup is not None else 3 * P
    run_proofs(fns, warm)
    elapsed = run_proofs_timed(fns, args.steps, pg, local)
    proof = set_proofs[0]
    assert proof is not None and all(p_ == proof for p_ in last if p_ is not None), \
        "provers disagree on the proof bytes"
    set_proofs_ok = all(set_proofs)
    # the single-trace window beside it (the round-4 headline's form): every proof from set 0
    sfns = [host_step(k, trace) for k in range(P)]
    single_s = None
    if not args.no_compare:
        single_s = run_proofs_timed(sfns, args.steps, pg, local)
        assert all(p_ == proof for p_ in last if p_ is not None), "provers disagree on the proof bytes"

    # ---- comparison legs (same provers, same count, outside the headline): the trace already in HBM
    # (zk_prove_device), and the host trace in pageable memory (runtime-staged copies)
    cmp_steps = max(2 * P, min(args.steps, 10))
    dev_s = pag_s = latency_ms = steady_s = mixed = None
    if not args.no_compare:
        steady_s = run_proofs_timed(fns, STEADY_PROOFS, pg, local)
        assert all(p_ == proof for p_ in last if p_ is not None), "provers disagree on the proof bytes"
        d_traces = [g.upload_trace(trace)[0] for g in provers]

        def dev_step(k):
            def f():
                last[k] = provers[k].prove_device(d_traces[k], n, pub, opts)[0]
            return f

        dfns = [dev_step(k) for k in range(P)]
        run_proofs(dfns, P)
        dev_s = run_proofs_timed(dfns, cmp_steps, pg, local)
        assert all(p_ == proof for p_ in last if p_ is not None), "device-resident proof differs"
        if not args.ab:
            pageable = np.array(trace)  # ordinary (pageable) host memory
            pfns = [host_step(k, pageable) for k in range(P)]
            run_proofs(pfns, P)
            pag_s = run_proofs_timed(pfns, cmp_steps, pg, local)
            assert all(p_ == proof for p_ in last if p_ is not None), "pageable-trace proof differs"
            del pageable
        vm_rec.update(vm_prove_leg(args, prog, src, w, proof, provers, opts, pg, local, rank))
        mixed = mixed_programs_leg(args, n, sets, provers, opts, pg, local)
    prog.close()
    for g in provers[1:]:
        g.close()
    if not args.no_compare:
        # latency of one prove() call alone on the GPU (host-resident trace), median of 5
        lat = []
        for _ in range(5):
            t1 = time.perf_counter()
            gpu.prove_host(trace, pub, opts)
            lat.append(time.perf_counter() - t1)
        latency_ms = 1e3 * sorted(lat)[len(lat) // 2]
    stages = gpu.stage_times()

    # one extra, untimed, profiled proof: per-kernel device time (HIP events on the prover stream), on the schedule the
    # timed proofs ran (it runs alone, which AUTO would give the latency schedule's smaller launches)
    gpu.set_upload_schedule(timed_sched)
    gpu.profile(True)
    gpu.prove_host(trace, pub, opts)
    kstats = gpu.kernel_stats()
    kops = gpu.kernel_ops()
    gpu.profile(False)
    gpu.set_upload_schedule(args.upload_schedule)
    upst = gpu.upload_stats()  # that proof's trace upload (sparse / narrow hints learned from the proofs before it)
    upload = {"mb_per_proof": round(upst["bytes"] / 2**20, 1), "full_trace_mb": round(28 * n * 16 / 2**20, 1),
              "sparse_cols": upst["sparse"], "narrow8_cols": upst["narrow8"], "narrow32_cols": upst["narrow32"],
              "derived_cols": upst["derived"],
              "schedule": {"timed_proofs": timed_sched, "profiled_proof": timed_sched,
                           "latency_leg": args.upload_schedule if args.upload_schedule != "auto" else "latency"}}

    verified = None
    if rank == 0 and not args.no_verify:
        import ctypes as C
        from oracle import oracle as orc
        orc.build()
        opub = orc.PubInputs()
        C.memmove(opub.program_hash, bytes(pub.program_hash), 32)
        C.memmove(opub.stack_outputs, bytes(pub.stack_outputs), 256)
        opub.lwe_size, opub.delta = pub.lwe_size, pub.delta
        verified = orc.verify(proof, opub, min_sec)[0] == 0
    from zkvm_amd.prover import verify as zk_verify
    zk_verified = zk_verify(proof, pub, min_sec)[0] == 0
    gpu.close()
    lifetime = None
    if not args.no_compare and not args.ab:
        lifetime = lifetime_leg(local, n, trace, pub, opts, proof)
    # every rank: its proof accepted by zk_verify; rank 0's workload (seed 1000) is a committed oracle pin, so its
    # proof must also equal the pin byte for byte (the other ranks' seeds have no pin)
    pin = pin_check(proof, find_pin(args.log_n, 1000 + rank, opts))
    all_verified = all_ranks_true(pg, zk_verified, local)
    cpu = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        # the reported CPU baseline: one single-thread oracle proof of the headline workload's own trace (input set
        # 0, the pinned configs[2] trace) -- its proof must be the GPU's bytes -- plus the bounded 2^18 samples
        cpu = cpu_headline(trace, pub, opts, proof, args.log_n)
        if args.cpu_sample:
            # (outside the default run) the bounded 2^cpu-log-n sample of earlier rounds, and the whole-host figure
            cpu["sample_small"] = cpu_baseline(args.cpu_log_n, args.config5, host_cores(args.cpu_cores))
            if "all_cores" in cpu["sample_small"]:
                cpu["all_cores"] = cpu["sample_small"].pop("all_cores")
    trace = None
    sets = None
    host.close()
    for hk in extra_hosts:
        hk.close()

    out = build_line(args, rank, world, n, elapsed, warm, opts, opts_str, min_sec, P, program_ops, padded_ops,
                     latency_ms, dev_s, pag_s, steady_s, cmp_steps, stages, kstats, kops, vm_rec, proof, verified,
                     zk_verified, pin, all_verified, lifetime, cpu) if rank == 0 else None
    if out is not None:
        out["gpu_max_hw_queues"] = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
        out["trace_upload"] = upload
        out["input_sets"] = {"count": S, "timed_proofs_rotate": True, "all_sets_proved_and_consistent": set_proofs_ok,
                             "single_trace_ms": round(1e3 * single_s / args.steps, 3) if single_s else None}
        out["runtime"] = native.runtime_info()
        if mixed is not None:
            mixed["vs_single_program"] = round(mixed["ms_per_proof"] / out["ms_per_step"], 4)
            mixed["vs_programs_alone"] = round(mixed["ms_per_proof"] / ((out["ms_per_step"] + mixed["pushadd_alone_ms"]) / 2), 4)
        out["mixed_programs"] = mixed
    if out is not None and world == 1 and not args.no_compare and not args.ab:
        q = queues_leg(args, P)
        out["queues_ab"] = q
        out["default_queues_ms"] = (out["ms_per_step"] if out["gpu_max_hw_queues"] == 4
                                    else q.get("ms_per_step"))

    # ---- multi-GPU: the north_star's ONE proof sharded by coset over all ranks (configs[3]) as a sub-record.  A
    # watchdog bounds it: should a collective never complete, rank 0 still prints the line (with the error) and
    # every rank exits, so the replica measurement above is never lost.
    if world > 1 and args.sharded_log_n:
        from zkvm_amd import native
        if native.device_count() > 0:
            done = threading.Event()

            def watchdog():
                # a hung collective: rank 0 still prints the line (the replica value stands, the sharded error is
                # in it), then every rank exits NON-zero so a stuck sharded proof is never mistaken for a clean run
                if not done.wait(SHARDED_TIMEOUT_S):
                    if out is not None:
                        out["sharded"] = {"error": f"the sharded proof did not finish within {SHARDED_TIMEOUT_S} s",
                                          "timed_out": True}
                        print(json.dumps(out), flush=True)
                    os._exit(3)

            threading.Thread(target=watchdog, daemon=True).start()
            try:
                rec = sharded_leg(args, args.sharded_log_n, world, rank, local, pg, steps=10, warmup=3)
                for k in ("pub", "proof", "n", "min_sec"):
                    rec.pop(k)
            except Exception as e:  # reported in the line; the replica value stands
                rec = {"error": repr(e)}
            done.set()
            if out is not None:
                out["sharded"] = rec

    if out is not None:
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.close()


SHARDED_TIMEOUT_S = 240


def lifetime_leg(local, n, trace, pub, opts, proof):
    """The reference builds its prover inside every vm::prove call (ExecutionProver::new, vm/src/lib.rs:24):
    cold_call_ms = zk_prover_create + the first proof (per-size tables) + zk_prover_destroy; pooled_call_ms = the same
    call shape through the process-wide pool (zk_prover_acquire + proof + zk_prover_release) once it holds a prover."""
    from zkvm_amd.prover import GpuProver
    from zkvm_amd.native import lib
    cold = []
    for _ in range(2):
        t0 = time.perf_counter()
        g = GpuProver(local, max_trace_len=n, max_blowup=opts.blowup_factor)
        p = g.prove_host(trace, pub, opts)[0]
        g.close()
        cold.append(1e3 * (time.perf_counter() - t0))
        assert p == proof
    pooled = []
    for _ in range(4):
        t0 = time.perf_counter()
        g = GpuProver(local, max_trace_len=n, max_blowup=opts.blowup_factor, pooled=True)
        p = g.prove_host(trace, pub, opts)[0]
        g.close()
        pooled.append(1e3 * (time.perf_counter() - t0))
        assert p == proof
    lib().zk_prover_pool_trim(local)
    return {"cold_call_ms": round(min(cold), 3), "cold_calls_ms": [round(x, 1) for x in cold],
            "pooled_call_ms": round(sorted(pooled[1:])[1], 3), "pooled_first_call_ms": round(pooled[0], 3),
            "call_shape": "one proof per call from the host-resident trace; cold: create + prove + destroy; pooled: "
                          "acquire + prove + release (median of 3 after the pool's first fill)"}


def queues_leg(args, P):
    """The headline configuration re-run in a child process at the OTHER hardware-queue count (GPU_MAX_HW_QUEUES
    4 <-> 16; HIP's default is 4 and this pool's boxes export 4): the design must not depend on a host raising it."""
    import subprocess
    other = "16" if os.environ.get("GPU_MAX_HW_QUEUES", "4") == "4" else "4"
    env = dict(os.environ, GPU_MAX_HW_QUEUES=other)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--no-cpu-baseline", "--no-verify", "--no-compare",
           "--sharded-log-n", "0", "--inflight", str(P), "--steps", str(args.steps), "--log-n", str(args.log_n)]
    if args.config5:
        cmd.append("--config5")
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        line = json.loads(r.stdout.strip().splitlines()[-1])
        return {"gpu_max_hw_queues": int(other), "ms_per_step": line["ms_per_step"], "value": line["value"],
                "inflight": P, "proof_matches_pin": line.get("proof_matches_pin")}
    except Exception as e:  # reported, never fatal for the headline
        return {"gpu_max_hw_queues": int(other), "error": repr(e)[:300]}


def mixed_programs_leg(args, n, sets, provers, opts, pg, local):
    """A server proving two programs of one trace length in turn (vm/src/lib.rs:13-29 serves any program): the timed
    proofs alternate the workload's cipher-mix input sets with a 2^log_n push/add program, whose column classes differ
    (push/add leaves s2..s15 and three opcode bits zero, the cipher mix s11..s15), P provers in flight as in the
    headline.  The column hints are keyed by (n, program hash), so neither program's hints void the other's proofs:
    `hint_redos` counts the proofs voided and redone in the window (0 expected); `ms_per_proof` sits beside the
    headline's ms_per_step (`vs_single_program`)."""
    from zkvm_amd.prover import HostTrace, Program, make_pub_inputs
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    src_b = ops_for_trace_len(args.log_n, "pushadd")
    wb = make_workload(src_b, seed=4242)
    prog_b = Program(src_b)
    if prog_b.trace_len != n:
        prog_b.close()
        return {"error": f"push/add program has trace length {prog_b.trace_len}, not {n}"}
    hb = HostTrace(n)
    tb, ob = prog_b.trace(wb.public, wb.secret, wb.server_key, wb.last_row, out=hb)
    pb = make_pub_inputs(prog_b.hash, ob, wb.server_key.lwe_size(), wb.server_key.parameters.delta)
    prog_b.close()
    mix = []
    for i in range(2 * len(sets)):  # cipher set 0, push/add, cipher set 1, push/add, ...
        mix.append(sets[i // 2] if i % 2 == 0 else (tb, pb))
    P = len(provers)
    nxt = [0]
    lock = threading.Lock()

    def mstep(k):
        def f():
            with lock:
                i = nxt[0] % len(mix)
                nxt[0] += 1
            provers[k].prove_host(mix[i][0], mix[i][1], opts)
        return f

    mfns = [mstep(k) for k in range(P)]
    run_proofs(mfns, 2 * P)  # both programs' hints learned
    redos0 = sum(g.proof_info()["hint_redos"] for g in provers)
    count = max(args.steps, 4 * P)
    ms = 1e3 * run_proofs_timed(mfns, count, pg, local) / count
    redos = sum(g.proof_info()["hint_redos"] for g in provers) - redos0
    info = provers[0].proof_info()

    # the push/add program alone, the same window: the mixed stream's cost against its two programs' own
    # (vs_programs_alone = mixed / mean(headline, push/add alone); 1.0 = alternating costs nothing)
    def bstep(k):
        return lambda: provers[k].prove_host(tb, pb, opts)

    bfns = [bstep(k) for k in range(P)]
    run_proofs(bfns, P)
    ms_b = 1e3 * run_proofs_timed(bfns, count, pg, local) / count
    hb.close()
    return {"ms_per_proof": round(ms, 3), "proofs": count, "hint_redos": redos,
            "hint_sets_per_prover": info["hint_sets"], "pushadd_alone_ms": round(ms_b, 3),
            "programs": f"cipher mix (configs[2], {len(sets)} input sets) alternating with a 2^{args.log_n}-step "
                        f"push/add program, P = {P} in flight"}


def vm_prove_leg(args, prog, src, w, proof, provers, opts, pg, local, rank):
    """vm::prove end to end with FRESH inputs per proof (vm/src/lib.rs:13-29; zk_vm_prove): each proof runs the
    host stack pass on its own inputs, uploads the machine states and inputs (~6 MB), writes the trace on the GPU and
    proves it -- no 448 MiB trace crosses PCIe.  P provers in flight, input sets dealt round-robin (set 0 is the
    replica workload, whose proof must equal the headline's)."""
    from zkvm_amd.prover import Program
    from zkvm_amd.workloads import make_workload
    sets = [(Program.encode_inputs(w.public, w.secret, w.server_key), w.last_row)]
    for k in range(3):
        wk = make_workload(src, seed=7000 + 16 * rank + k)
        sets.append((Program.encode_inputs(wk.public, wk.secret, wk.server_key), wk.last_row))
    P = len(provers)
    nxt = [0]
    lock = threading.Lock()

    def vstep(k):
        def f():
            with lock:
                i = nxt[0] % len(sets)
                nxt[0] += 1
            prog.prove_device(provers[k], sets[i][0], sets[i][1], opts)
        return f

    vfns = [vstep(k) for k in range(P)]
    # the first call on a device uploads the program (code, sponge columns) and builds its preprocessed columns
    # (the program-only columns' coefficients and LDE): once per program, like Program::compile
    t0 = time.perf_counter()
    prog.prove_device(provers[0], sets[0][0], sets[0][1], opts)
    first_ms = 1e3 * (time.perf_counter() - t0)
    run_proofs(vfns, P)
    count = max(args.steps, 2 * P)
    vm_s = run_proofs_timed(vfns, count, pg, local)
    lat = []
    for _ in range(3):
        t0 = time.perf_counter()
        _, _, p0 = prog.prove_device(provers[0], sets[0][0], sets[0][1], opts)
        lat.append(time.perf_counter() - t0)
    return {"vm_prove_ms": round(1e3 * vm_s / count, 3), "vm_prove_proofs": count, "vm_prove_input_sets": len(sets),
            "vm_prove_first_call_ms": round(first_ms, 3),
            "vm_prove_latency_ms": round(1e3 * sorted(lat)[1], 3), "vm_prove_same_proof": p0 == proof,
            "vm_prove_timed_region": "zk_vm_prove: host stack pass + state/input upload + GPU trace + proof, fresh "
                                     "inputs per proof, P in flight"}


def build_line(args, rank, world, n, elapsed, warm, opts, opts_str, min_sec, P, program_ops, padded_ops, latency_ms,
               dev_s, pag_s, steady_s, cmp_steps, stages, kstats, kops, vm_rec, proof, verified, zk_verified, pin,
               all_verified, lifetime, cpu):
    """rank 0's JSON line (the driver's contract) from the measurements of main()."""
    dom = max(kstats.items(), key=lambda kv: kv[1][0])
    name, (tot_ms, launches, tot_bytes) = dom
    avg_ms = tot_ms / launches
    achieved = tot_bytes / (tot_ms / 1e3) / 1e9
    prove_total_ms = sum(v[0] for v in kstats.values())
    # the committed PMC profiles are taken at 2^20 (tools/gpu_profile.sh): other sizes report no traffic
    PROFILED_LOG_N = 20
    tr = pmc_traffic(name, args.config5) if args.log_n == PROFILED_LOG_N else None
    # What bounds the kernel is VALU issue (the f128 carry chains' SGPR port), not HBM: the line
    # says so in `bound`, keeps the contract's HBM figures (achieved / peak / frac: algorithmic bytes per launch over
    # the launch time, the BASELINE metric's roofline) and the measured traffic ratio beside it, and gives the binding
    # resource's hardware utilisation as `compute_frac` (SQ_INSTS_VALU over the SIMDs' issue slots, profiles/).
    hw = pmc_valu(name) if args.log_n == PROFILED_LOG_N else None
    roofline = {"bound": "valu-issue", "kernel": name,
                "bound_note": "integer-VALU issue (f128 carry chains); achieved/peak/frac are the HBM roofline of the "
                              "contract, compute_frac the hardware VALU issue-slot utilisation of the same kernel",
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "hbm_frac": round(achieved / HBM_PEAK_GBS, 4),
                "compute_frac": hw["slot_util"] if hw else None,
                "compute_unit": "VALU issue slots: SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 2)",
                "traffic": tr["per_launch_bytes"] if tr else None,
                "traffic_ratio": tr["traffic_ratio"] if tr else None, "traffic_source": tr,
                "avg_launch_ms": round(avg_ms, 4), "launches_per_step": launches,
                "alg_bytes_per_launch": tot_bytes / launches,
                "kernel_share_of_device_time": round(tot_ms / prove_total_ms, 3)}
    if name in kops:
        # the same launches against this build's own field-op costs: their algorithmic f128 multiplies and add/subs
        # priced at the measured throughput of this library's fe_mul / fe_add / fe_sub (a self-referential floor:
        # how close the kernel is to its own arithmetic, not to the hardware -- compute_frac is the hardware figure).
        # Multiplies count in fe_mul-equivalents (a W-set multiply 80/113: kernels.hip uniform_mul_discount)
        muls, addsubs = kops[name]
        floor_ms = 1e3 * (muls / FE_MUL_PEAK + addsubs / (0.5 * FE_ADD_PEAK + 0.5 * FE_SUB_PEAK))
        roofline["valu_vs_build_fe_ops"] = {
            "basis": "this build's measured fe_mul / fe_add / fe_sub throughput (tools/ubench/mul_ubench.hip)",
            "fe_mul_equiv_per_launch": muls / launches, "fe_addsub_per_launch": addsubs / launches,
            "achieved_fe_mul_per_s": round(muls / (tot_ms / 1e3), 1), "peak_fe_mul_per_s": FE_MUL_PEAK,
            "floor_ms_per_launch": round(floor_ms / launches, 4), "frac_vs_build_fe_mul_cost": round(floor_ms / tot_ms, 4)}
    roofline["valu_hw"] = hw
    value = world * n * args.steps / elapsed
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "trace-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": warm, "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f128", "data": "synthetic (seeded VM trace)",
        "config": {"workload": f"configs[{4 if args.config5 else 2}]: 2^{args.log_n}-step READ2/ADD2/SMUL cipher-mix program, "
                               f"full prove from the host-resident trace" +
                               (" at 128-bit conjectured security" if args.config5 else ""),
                   "trace_len": n, "trace_width": 28, "lde_len": n * opts.blowup_factor,
                   "program_ops": program_ops, "padded_ops": padded_ops,
                   "options": opts_str, "timed_region": "zk_prove_columns: page-locked host trace -> proof bytes",
                   "parallelism": f"independent proofs, {P} in flight per GPU, x{world} GPUs",
                   "host_numa_node": HOST["numa_node"]},
        "security_bits_checked": min_sec,
        "latency_ms": round(latency_ms, 3) if latency_ms is not None else None,
        "device_resident_ms": round(1e3 * dev_s / cmp_steps, 3) if dev_s is not None else None,
        "pageable_host_ms": round(1e3 * pag_s / cmp_steps, 3) if pag_s is not None else None,
        "steady_state_ms": round(1e3 * steady_s / STEADY_PROOFS, 3) if steady_s is not None else None,
        "roofline": roofline, "cpu_baseline": cpu,
        "stage_ms": {k: round(v, 3) for k, v in stages.items()},
        "kernel_ms": {k: round(v[0], 3) for k, v in sorted(kstats.items(), key=lambda kv: -kv[1][0])},
        "kernel_launches": {k: v[1] for k, v in kstats.items()},
        "kernel_alg_bytes": {k: v[2] for k, v in kstats.items()},
        "vm": vm_rec,
        "proof_bytes": len(proof), "proof_verified_by_oracle": verified, "proof_verified_by_zk_verify": zk_verified,
        "proof_matches_pin": pin["proof_matches_pin"] if pin else None, "pin": pin["pin"] if pin else None,
        "all_ranks_verified_by_zk_verify": all_verified,
        "prover_lifetime": lifetime,
    }
    return out


def sharded_leg(args, log_n, world, rank, local, pg, steps, warmup, config5=False):
    """One 2^log_n proof per step with the LDE domain sharded by coset over all ranks (zk_prove_sharded over
    RCCL): every rank proves the same trace.  Timed twice: from the page-locked host trace (the reference's call
    shape; each rank uploads and interpolates its 1/G of the columns) and from a trace already in every rank's
    HBM.  Returns (on every rank) the step times and stage split."""
    from zkvm_amd.prover import HostTrace, Program, ProofOptions, make_pub_inputs
    from zkvm_amd.sharded import ShardedProver
    from zkvm_amd.workloads import make_workload, ops_for_trace_len
    src = ops_for_trace_len(log_n, "cipher")
    w = make_workload(src, seed=1000)  # the same trace on every rank: one proof
    t0 = time.perf_counter()
    prog = Program(src)
    host = HostTrace(prog.trace_len)
    trace, outputs = prog.trace(w.public, w.secret, w.server_key, w.last_row, out=host)
    h = prog.hash
    n = trace.shape[1]
    log(f"[rank {rank}] sharded VM trace: n={n} ({time.perf_counter() - t0:.1f} s)")
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    opts = ProofOptions(43, 8, 0, 2, 8, 127) if config5 else ProofOptions()
    if REHEARSE and world > 1:
        # several ranks on one GPU: exchanges through host memory over the TCP host group (RCCL refuses a
        # communicator with two ranks on one device)
        sp = ShardedProver.host(rank, world, pg.exchange_fn(), local, n)
    else:
        # RCCL from the library's own runtime (native.runtime_info()["rccl"]); the id travels over the host group
        uid = ShardedProver.unique_id() if rank == 0 else None
        if pg is not None:
            uid = pg.broadcast(uid, src=0)
        sp = ShardedProver.rccl(rank, world, uid, local, n)
    last = {}

    def step_host():
        last["proof"] = sp.prove(trace, pub, opts)[0]

    elapsed = timed_loop(step_host, steps, warmup, pg, local)
    stages = sp.stage_times()
    xchg_host = sp.exchange_stats(exposed=True)
    sp.upload_trace(trace)

    def step_dev():
        last["proof_dev"] = sp.prove(None, pub, opts, n=n)[0]

    elapsed_dev = timed_loop(step_dev, steps, 1, pg, local)
    xchg_dev = sp.exchange_stats(exposed=True)
    # vm::prove sharded (zk_vm_prove_sharded): every rank writes the trace into its own HBM from the program and the
    # inputs (its host runs the stack pass), then the same sharded proof -- no trace over PCIe or xGMI
    inp = Program.encode_inputs(w.public, w.secret, w.server_key)

    def step_vm():
        last["proof_vm"] = sp.prove_program(prog, inp, w.last_row, opts)[2]

    elapsed_vm = timed_loop(step_vm, steps, 1, pg, local)
    stages_vm = sp.stage_times()
    prog.close()
    proof = last["proof"]
    same = last["proof_dev"] == proof and last["proof_vm"] == proof
    # self-check on every rank: the RCCL proof equals the committed oracle pin of this exact workload (configs[3]:
    # c3_cipher_2p22, seed 1000) and zk_verify accepts it; all ranks must agree
    from zkvm_amd.prover import verify as zk_verify
    pin = pin_check(proof, find_pin(log_n, 1000, opts))
    ok_verify = zk_verify(proof, pub, 128 if config5 else 95)[0] == 0
    ok_pin = pin["proof_matches_pin"] if pin else True
    all_verify = all_ranks_true(pg, ok_verify and same, local)
    all_pin = all_ranks_true(pg, ok_pin, local) if pin else None
    sp.close()
    del trace
    host.close()
    return {"workload": f"configs[{4 if config5 else 3}]: one 2^{log_n}-step cipher-mix proof, LDE domain sharded by coset",
            "timed_region": "zk_prove_sharded from the page-locked host trace on every rank",
            "n_ranks": world, "steps": steps, "warmup": warmup, "ms_per_proof": round(1e3 * elapsed / steps, 3),
            "trace_steps_per_s": round(n * steps / elapsed, 1), "scaling": "strong",
            "device_resident_ms_per_proof": round(1e3 * elapsed_dev / steps, 3),
            "vm_prove_ms_per_proof": round(1e3 * elapsed_vm / steps, 3),
            "vm_prove_stage_ms": {k: round(v, 3) for k, v in stages_vm.items()},
            "device_resident_and_vm_prove_same_proof": same,
            "stage_ms": {k: round(v, 3) for k, v in stages.items()}, "proof_bytes": len(proof),
            "pin": pin["pin"] if pin else None, "proof_matches_pin": all_pin,
            "all_ranks_verified_by_zk_verify": all_verify,
            "exchange": exchange_record(xchg_host), "exchange_device_resident": exchange_record(xchg_dev),
            "model": model_record(log_n, world, config5, {"host": 1e3 * elapsed / steps,
                                                          "device": 1e3 * elapsed_dev / steps,
                                                          "vm": 1e3 * elapsed_vm / steps}),
            "pub": pub, "proof": proof, "n": n, "min_sec": 128 if config5 else 95}


SHARD_MODEL = "profiles/r06fin_shard_schedule_2p22.json"


def model_record(log_n, world, config5, measured):
    """The one-GPU replay model's per-rank projection for this world size (tools/shard_model.py --schedule, committed
    under profiles/) beside the measured ms per proof of each trace source, so a multi-GPU run checks the model."""
    path = Path(__file__).resolve().parent / SHARD_MODEL
    if config5 or not path.exists():
        return None
    d = json.loads(path.read_text())
    if d.get("log_n") != log_n:
        return None
    out = {"source": SHARD_MODEL}
    if REHEARSE:  # ranks sharing one GPU over TCP: the comparison is not a measurement of the model
        out["rehearsal"] = True
    for kind, ms in measured.items():
        pr = d.get("projection", {}).get(kind, {}).get(str(world))
        if pr:
            out[kind] = {"measured_ms": round(ms, 3), "modelled_per_rank_ms": pr["per_rank_ms"],
                         "measured_over_modelled": round(ms / pr["per_rank_ms"], 3)}
    return out


def exchange_record(stats):
    """Per collective of the last sharded proof on rank 0: ms (HIP events around it on the exchange stream, waiting
    for peers included), exposed ms (how long the compute stream waited for it, when the stats carry it), MB received
    from the other ranks, calls, and the effective receive rate."""
    out = {}
    for name, v in stats.items():
        ms, by, calls = v[0], v[1], v[2]
        out[name] = {"ms": round(ms, 3), "mb_received": round(by / 1e6, 3), "calls": calls,
                     "gb_per_s": round(by / 1e6 / ms, 2) if ms > 0 else None}
        if len(v) > 3:
            out[name]["exposed_ms"] = round(v[3], 3)
    tot_ms = sum(v[0] for v in stats.values())
    tot_b = sum(v[1] for v in stats.values())
    out["total"] = {"ms": round(tot_ms, 3), "mb_received": round(tot_b / 1e6, 3),
                    "gb_per_s": round(tot_b / 1e6 / tot_ms, 2) if tot_ms > 0 else None}
    if any(len(v) > 3 for v in stats.values()):
        out["total"]["exposed_ms"] = round(sum(v[3] for v in stats.values() if len(v) > 3), 3)
    return out


def run_sharded(args):
    world, rank, local, pg = setup_dist(args.gpus)
    from zkvm_amd import native
    from zkvm_amd.workloads import ops_for_trace_len, padded_length
    native.lib()
    warm = args.warmup if args.warmup is not None else 3
    rec = sharded_leg(args, args.log_n, world, rank, local, pg, args.steps, warm, args.config5)
    verified = None
    if rank == 0 and not args.no_verify:
        import ctypes as C
        from oracle import oracle as orc
        orc.build()
        pub = rec["pub"]
        opub = orc.PubInputs()
        C.memmove(opub.program_hash, bytes(pub.program_hash), 32)
        C.memmove(opub.stack_outputs, bytes(pub.stack_outputs), 256)
        opub.lwe_size, opub.delta = pub.lwe_size, pub.delta
        verified = orc.verify(rec["proof"], opub, rec["min_sec"])[0] == 0
    if rank == 0:
        src = ops_for_trace_len(args.log_n, "cipher")
        n = rec["n"]
        out = {
            "metric": METRIC, "value": rec["trace_steps_per_s"], "unit": "trace-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": warm, "ms_per_step": rec["ms_per_proof"],
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f128",
            "data": "synthetic (seeded VM trace)",
            "config": {"workload": rec["workload"], "trace_len": n, "trace_width": 28, "lde_len": 8 * n,
                       "program_ops": sum(1 for ln in src.splitlines() if ln.split("#")[0].strip()),
                       "padded_ops": padded_length(src),
                       "options": ("ProofOptions(43, 8, 0, Quadratic, 8, 127)" if args.config5
                                   else "ProofOptions(32, 8, 0, None, 8, 127)"),
                       "parallelism": f"coset-sharded x{world} (RCCL all-to-all / all-gather)",
                       "timed_region": rec["timed_region"]},
            "device_resident_ms": rec["device_resident_ms_per_proof"],
            "vm_prove_ms": rec["vm_prove_ms_per_proof"],
            "device_resident_and_vm_prove_same_proof": rec["device_resident_and_vm_prove_same_proof"],
            "roofline": None, "cpu_baseline": None, "stage_ms": rec["stage_ms"],
            "proof_bytes": rec["proof_bytes"], "proof_verified_by_oracle": verified,
            "pin": rec["pin"], "proof_matches_pin": rec["proof_matches_pin"],
            "all_ranks_verified_by_zk_verify": rec["all_ranks_verified_by_zk_verify"],
            "exchange": rec["exchange"], "exchange_device_resident": rec["exchange_device_resident"],
        }
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.close()


if __name__ == "__main__":
    main()
