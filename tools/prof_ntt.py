"""Drive the NTT kernels alone (zk_diag_ntt: 28 polys of 2^LOG, forward over a coset, then inverse)
for counter collection:  rocprofv3 --pmc SQ_... -- python3 tools/prof_ntt.py [LOG]"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "encrypt-zkvm_amd")]
from zkvm_amd import native  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n, batch = 1 << log_n, 28
vals = np.random.default_rng(1).integers(0, 2**63, size=(batch * n, 2), dtype=np.uint64)
out = np.empty_like(vals)
three = (3).to_bytes(16, "little")
for _ in range(2):
    native.check(native.lib().zk_diag_ntt(0, vals.ctypes.data, n, batch, 0, three, out.ctypes.data))
    native.check(native.lib().zk_diag_ntt(0, vals.ctypes.data, n, batch, 1, None, out.ctypes.data))
print("ok")
