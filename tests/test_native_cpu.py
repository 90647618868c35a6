"""CPU-side checks of the product library (no GPU needed).

  * libzkvm_gpu.so loads and exports every function include/zkvm_gpu.h declares;
  * the exact device multiply algorithm (fe_mul_limbs, run on the host) agrees with big-int
    arithmetic, including carry/borrow edge cases of the two-fold reduction;
  * the host BLAKE3 used by the transcript agrees with the oracle's;
  * the product VM (zk_vm_trace) reproduces the oracle VM's traces and error texts bit for bit.
"""
import ctypes as C
import random
import re
from pathlib import Path

import numpy as np
import pytest

from zkvm_amd import native
from zkvm_amd.prover import bytes_elems, elems_bytes, vm_trace
from zkvm_amd.workloads import LR_PROGRAM, ServerKey, cipher_mix_program, make_workload, push_add_program

ROOT = Path(__file__).resolve().parent.parent
P = 2**128 - 45 * 2**40 + 1


def header_functions():
    text = (ROOT / "include" / "zkvm_gpu.h").read_text()
    return sorted(set(re.findall(r"\b(zk_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_header_symbols():
    L = native.lib()
    declared = header_functions()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(L, name), f"{name} declared in include/zkvm_gpu.h but not exported"
    assert set(native.EXPORTED) <= set(declared)


def test_null_arguments_refused_without_gpu():
    """The setters and the prove entry points check their arguments before touching a device: null provers, traces
    and columns are refused with ZK_ERR_INVALID_ARG (no GPU needed to reach the checks)."""
    L = native.lib()
    assert L.zk_prover_set_upload_schedule(None, 0) == native.ZK_ERR_INVALID_ARG
    assert L.zk_prover_profile(None, 1) == native.ZK_ERR_INVALID_ARG
    # the prove entry points check their pointers before the prover: a null trace, a null column among 28
    plen = C.c_size_t(0)
    assert L.zk_prove(None, None, 16, None, None, None, C.byref(plen)) == native.ZK_ERR_INVALID_ARG
    cols = (C.c_void_p * 28)(*([C.c_void_p(1)] * 27 + [None]))
    assert L.zk_prove_columns(None, cols, 16, None, None, None, C.byref(plen)) == native.ZK_ERR_INVALID_ARG
    assert L.zk_prove_columns(None, None, 16, None, None, None, C.byref(plen)) == native.ZK_ERR_INVALID_ARG
    assert L.zk_vm_prove(None, None, None, 0, None, 0, 5, 16, None, None, None, C.byref(plen), None, None) \
        == native.ZK_ERR_INVALID_ARG


def edge_values():
    vals = [0, 1, 2, P - 1, P - 2, 2**64 - 1, 2**64, 2**127, P - 2**64, 45 * 2**40, 2**96 - 1, 2**128 - 45 * 2**40]
    vals += [P - 1 - (1 << k) for k in range(0, 127, 7)]
    return vals


def test_device_mul_algorithm_on_host():
    rnd = random.Random(3)
    a = edge_values() + [rnd.randrange(P) for _ in range(2000)]
    b = list(reversed(edge_values())) + [rnd.randrange(P) for _ in range(2000)]
    a, b = a + b, b + a
    out = C.create_string_buffer(16 * len(a))
    native.lib().zk_diag_mul_limbs_host(elems_bytes(a), elems_bytes(b), out, len(a))
    got = bytes_elems(out.raw)
    for x, y, r in zip(a, b, got):
        assert r == x * y % P, (x, y)


def test_lazy_dot_product_on_host():
    """acc288: sums of unreduced 256-bit products with one final reduction (constraint evaluator, DEEP)."""
    rnd = random.Random(11)
    cases = [[P - 1] * 40, [0] * 3, edge_values()] + [[rnd.randrange(P) for _ in range(k)] for k in (1, 2, 7, 28, 300)]
    for a in cases:
        b = list(reversed(a)) if len(a) > 3 else a
        out = C.create_string_buffer(16)
        native.lib().zk_diag_dot_host(elems_bytes(a), elems_bytes(b), len(a), out)
        assert bytes_elems(out.raw)[0] == sum(x * y for x, y in zip(a, b)) % P


def test_host_blake3_matches_oracle(oracle):
    for n in (0, 1, 40, 63, 64, 65, 448, 1024, 1025, 2048, 4100):
        data = bytes((7 * i + 3) % 256 for i in range(n))
        out = C.create_string_buffer(32)
        native.lib().zk_diag_blake3_host(data, n, out)
        assert out.raw == oracle.blake3(data)


@pytest.mark.parametrize("source", [LR_PROGRAM, "push.5\npush.3\nadd", push_add_program(50), cipher_mix_program(20)[0]])
def test_vm_trace_matches_oracle(oracle, source):
    w = make_workload(source, seed=9)
    trace, outputs, h = vm_trace(source, w.public, w.secret, w.server_key, w.last_row)
    codes, values, oh = oracle.program_compile(source)
    otrace, oout = oracle.processor_trace(codes, values, w.public, w.secret, last_row=w.last_row)
    assert h == oh
    assert outputs == oout
    assert trace.shape == otrace.shape
    assert np.array_equal(trace, otrace)


@pytest.mark.parametrize("source,code", [("push.1\nad", native.ZK_ERR_PROGRAM), ("push.2\nmul", native.ZK_ERR_STACK),
                                         ("read", native.ZK_ERR_STACK), ("\n".join(["push.1"] * 17), native.ZK_ERR_STACK)])
def test_vm_errors_match_oracle(oracle, source, code):
    sk = ServerKey(seed=1)
    with pytest.raises(native.ZkError) as e:
        vm_trace(source, [], [], sk, [1] * 28)
    assert e.value.code == code
    with pytest.raises(oracle.OracleError) as oe:
        codes, values, _ = oracle.program_compile(source)
        oracle.processor_trace(codes, values)
    assert str(oe.value) in str(e.value)


def test_reference_vm_program_output():
    """The VM half of vm/src/lib.rs:47-99 (test_prove): read2 / read / sadd / push.1 / push.2 / add / smul
    with a = 1, x = Enc(2) decrypts to (a + x) * 3 on the top of the stack."""
    from zkvm_amd.workloads import LweParameters, rand_field
    src = "read2\nread\nsadd\npush.1\npush.2\nadd\nsmul\n"
    sk = ServerKey(LweParameters(8, 128, 4, 2.412_390_240_121_573e-5), seed=99)
    x = sk.encrypt(2)
    last_row = [rand_field(np.random.default_rng(5), lo=1) for _ in range(28)]
    trace, output, h = vm_trace(src, [1, 3], [x], sk, last_row)
    assert trace.shape[0] == 28 and sk.decrypt(output[:5]) == 9


def _in_fresh_process(code: str) -> dict:
    import json
    import subprocess
    import sys
    pre = f"import json, sys; sys.path[:0] = [{str(ROOT)!r}, {str(ROOT / 'encrypt-zkvm_amd')!r}]\n"
    r = subprocess.run([sys.executable, "-c", pre + code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_one_hip_runtime_the_one_the_library_links():
    """native.lib() in a torch-free process maps exactly one libamdhip64 -- /opt/rocm's, the RUNPATH the library was
    linked with (what a Rust host would load) -- and refuses a later `import torch`, which would map torch's bundled
    copy as a second runtime."""
    out = _in_fresh_process(
        "from zkvm_amd import native\n"
        "native.lib()\n"
        "info = native.runtime_info()\n"
        "hips = native.mapped_files('libamdhip64.so')\n"
        "try:\n"
        "    import torch\n"
        "    refused = False\n"
        "except ImportError:\n"
        "    refused = True\n"
        "print(json.dumps({'info': info, 'hips': hips, 'after': native.mapped_files('libamdhip64.so'),"
        " 'refused': refused}))\n")
    assert len(out["hips"]) == 1 and out["hips"] == out["after"]
    assert out["info"]["hip_runtime"] == out["hips"][0]
    assert out["info"]["hip_runtime"].startswith("/opt/rocm") and "/torch/" not in out["info"]["hip_runtime"]
    assert out["info"]["rccl"].startswith("/opt/rocm")
    assert out["info"]["hip_runtime_version"] >= 70200000 and out["info"]["rccl_version"] > 0
    assert out["refused"] and not out["info"]["torch_loaded_first"]


def test_torch_first_gives_one_shared_runtime():
    """A host that imports torch first: the library shares torch's runtime (still one mapping), and says so."""
    out = _in_fresh_process(
        "import torch\n"
        "from zkvm_amd import native\n"
        "native.lib()\n"
        "print(json.dumps({'info': native.runtime_info(), 'hips': native.mapped_files('libamdhip64.so')}))\n")
    assert len(out["hips"]) == 1 and out["info"]["hip_runtime"] == out["hips"][0]
    assert out["info"]["torch_loaded_first"]
