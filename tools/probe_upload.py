"""Host -> device copy rates on the GPU box for a 28 x 2^20 f128 trace (448 MiB): one copy vs per-column copies,
one vs two copy streams, page-locked (zk_host_alloc) vs pageable source.  Usage: python3 tools/probe_upload.py
"""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "encrypt-zkvm_amd"))

from zkvm_amd.prover import HostTrace  # noqa: E402

hip = C.CDLL("libamdhip64.so")
vp, sz = C.c_void_p, C.c_size_t
hip.hipMalloc.argtypes = [C.POINTER(vp), sz]
hip.hipMemcpyAsync.argtypes = [vp, vp, sz, C.c_int, vp]
hip.hipStreamCreateWithFlags.argtypes = [C.POINTER(vp), C.c_uint]
hip.hipStreamSynchronize.argtypes = [vp]
hip.hipDeviceSynchronize.argtypes = []


def main():
    n = 1 << 20
    nbytes = 28 * n * 16
    d = vp()
    assert hip.hipMalloc(C.byref(d), nbytes) == 0
    streams = [vp() for _ in range(4)]
    for s in streams:
        assert hip.hipStreamCreateWithFlags(C.byref(s), 1) == 0  # hipStreamNonBlocking, as the prover's
    ht = HostTrace(n)
    ht.array[:] = 7
    pg = np.full((28, n, 2), 7, dtype=np.uint64)
    for name, base in (("pinned", ht.array.ctypes.data), ("pageable", pg.ctypes.data)):
        for chunks, nst in ((1, 1), (28, 1), (28, 2), (28, 4), (112, 2), (112, 4)):
            per = nbytes // chunks
            best, times = 1e9, []
            for _ in range(4):
                hip.hipDeviceSynchronize()
                t0 = time.perf_counter()
                for k in range(chunks):
                    assert hip.hipMemcpyAsync(vp(d.value + k * per), vp(base + k * per), per, 1, streams[k % nst]) == 0
                for s in streams[:nst]:
                    hip.hipStreamSynchronize(s)
                times.append(time.perf_counter() - t0)
                best = min(best, times[-1])
            print(f"{name:8s} chunks={chunks:3d} streams={nst}: {best * 1e3:7.2f} ms  {nbytes / best / 1e9:6.1f} GB/s  "
                  f"(all: {' '.join(f'{1e3 * t:.2f}' for t in times)})", flush=True)
    ht.close()


if __name__ == "__main__":
    main()
