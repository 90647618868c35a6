"""Upload rate of a page-locked 2^20 trace inside a prover process: raw per-column copies into the prover's trace
buffer before and after proofs, then host-resident proofs one at a time (stage split), for rocprofv3 kernel /
copy traces of the upload overlap.  python3 tools/probe_host_prove.py [proofs] [pageable]
"""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "encrypt-zkvm_amd"))

from zkvm_amd.prover import GpuProver, HostTrace, ProofOptions, make_pub_inputs, vm_trace  # noqa: E402
from zkvm_amd.workloads import make_workload, ops_for_trace_len, trace_length  # noqa: E402

hip = C.CDLL("libamdhip64.so")
vp, sz = C.c_void_p, C.c_size_t
hip.hipMemcpyAsync.argtypes = [vp, vp, sz, C.c_int, vp]
hip.hipStreamCreateWithFlags.argtypes = [C.POINTER(vp), C.c_uint]
hip.hipStreamSynchronize.argtypes = [vp]


def raw_copies(dst, src, n, st, label):
    col = n * 16
    for rep in range(3):
        t0 = time.perf_counter()
        for c in range(28):
            assert hip.hipMemcpyAsync(vp(dst + c * col), vp(src + c * col), col, 1, st) == 0
        hip.hipStreamSynchronize(st)
        dt = time.perf_counter() - t0
        print(f"{label} rep {rep}: {1e3 * dt:.2f} ms {28 * col / dt / 1e9:.1f} GB/s", flush=True)


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    src = ops_for_trace_len(20, "cipher")
    w = make_workload(src, seed=1000)
    n = trace_length(src)
    ht = HostTrace(n)
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row, out=ht)
    if len(sys.argv) > 2 and sys.argv[2] == "pageable":
        trace = np.array(trace)
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    g = GpuProver(0, max_trace_len=n)
    st = vp()
    assert hip.hipStreamCreateWithFlags(C.byref(st), 1) == 0
    raw_copies(g.trace_buffer(), trace.ctypes.data, n, st, "before proofs")
    for _ in range(3):
        g.prove_host(trace, pub, ProofOptions())
    raw_copies(g.trace_buffer(), trace.ctypes.data, n, st, "after proofs")
    for _ in range(k):
        t0 = time.perf_counter()
        g.prove_host(trace, pub, ProofOptions())
        s = g.stage_times()
        print(f"{1e3 * (time.perf_counter() - t0):.2f} ms  trace_commit {s['trace_commit']:.2f} ms", flush=True)
    raw_copies(g.trace_buffer(), trace.ctypes.data, n, st, "at the end")
    g.close()


if __name__ == "__main__":
    main()
