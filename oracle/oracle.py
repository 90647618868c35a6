"""ctypes loader for the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker, never as the product path.
Parity unpinned at the winterfell boundary -- see oracle/oracle.h and DESIGN.md.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
# ORACLE_LIB selects another build of the same sources (tests/test_asan.py: the sanitizer build)
LIB_PATH = Path(os.environ.get("ORACLE_LIB", HERE / "liboracle.so"))
P = 2**128 - 45 * 2**40 + 1
MAX_COLS, MAX_TCONS, MAX_ASSERTS, MAX_CCOLS, MAX_FRI, MAX_REM, MAX_Q = 32, 32, 32, 16, 16, 256, 255


class Options(C.Structure):
    _fields_ = [(f, C.c_uint32) for f in
                ("num_queries", "blowup", "grinding", "field_extension", "fri_folding", "fri_rem_max_deg")]


class PubInputs(C.Structure):
    _fields_ = [("program_hash", C.c_uint8 * 32), ("stack_outputs", C.c_uint8 * 256),
                ("lwe_size", C.c_uint32), ("delta", C.c_uint32)]


class Record(C.Structure):
    _fields_ = [
        ("trace_len", C.c_uint32), ("lde_len", C.c_uint32), ("width", C.c_uint32), ("num_ccols", C.c_uint32),
        ("num_fri_layers", C.c_uint32), ("remainder_len", C.c_uint32), ("num_positions", C.c_uint32),
        ("_pad", C.c_uint32),
        ("trace_root", C.c_uint8 * 32),
        ("coeff_t", C.c_uint8 * (16 * MAX_TCONS)), ("coeff_b", C.c_uint8 * (16 * MAX_ASSERTS)),
        ("constraint_root", C.c_uint8 * 32), ("z", C.c_uint8 * 16),
        ("ood_trace_z", C.c_uint8 * (16 * MAX_COLS)), ("ood_trace_zg", C.c_uint8 * (16 * MAX_COLS)),
        ("ood_constraints", C.c_uint8 * (16 * MAX_CCOLS)),
        ("deep_t", C.c_uint8 * (16 * MAX_COLS)), ("deep_c", C.c_uint8 * (16 * MAX_CCOLS)),
        ("fri_roots", C.c_uint8 * (32 * MAX_FRI)), ("fri_alphas", C.c_uint8 * (16 * MAX_FRI)),
        ("remainder", C.c_uint8 * (16 * MAX_REM)), ("remainder_commitment", C.c_uint8 * 32),
        ("pow_nonce", C.c_uint64), ("positions", C.c_uint64 * (MAX_Q + 1)),
    ]


class Dump(C.Structure):
    _fields_ = [(f, C.c_void_p) for f in ("trace_polys", "trace_lde", "trace_leaves", "composition",
                                          "comp_polys", "comp_lde", "deep", "fri_layer1")]


def build(force: bool = False) -> Path:
    if "ORACLE_LIB" in os.environ:
        return LIB_PATH
    if force or not LIB_PATH.exists() or any(
            p.stat().st_mtime > LIB_PATH.stat().st_mtime for p in HERE.glob("*.[ch]")):
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        vp, sz, u32, u64, u8p = C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint64, C.c_char_p
        for name in ("or_fadd", "or_fsub", "or_fmul", "or_fexp"):
            getattr(L, name).argtypes = [vp, vp, vp]
        L.or_finv.argtypes = [vp, vp]
        L.or_e2_mul.argtypes = [vp, vp, vp]
        L.or_e2_inv.argtypes = [vp, vp]
        L.or_root_of_unity.argtypes = [u32, vp]
        L.or_eval_coset.argtypes = [vp, sz, sz, vp, vp]
        L.or_interp_coset.argtypes = [vp, sz, vp]
        L.or_blake3.argtypes = [vp, sz, vp]
        L.or_blake3_merge.argtypes = [vp, vp, vp]
        L.or_merkle_root.argtypes = [vp, sz, vp]
        L.or_rescue_apply_round.argtypes = [vp, C.c_uint8, C.c_uint8, u64]
        L.or_rescue_ark.argtypes = [u32, u32, vp]
        L.or_program_compile.argtypes = [u8p, vp, vp, sz, C.POINTER(sz), vp, vp, sz]
        L.or_processor_trace.argtypes = [vp, vp, sz, vp, sz, vp, sz, u32, u32, vp, vp, sz, C.POINTER(sz), vp,
                                         vp, sz]
        L.or_air_periodic_row.argtypes = [u32, vp]
        L.or_air_eval_transition.argtypes = [vp, vp, vp, u32, u32, vp]
        L.or_prove.argtypes = [vp, sz, C.POINTER(Options), C.POINTER(PubInputs), vp, C.POINTER(sz),
                               C.POINTER(Record), C.POINTER(Dump)]
        L.or_verify.argtypes = [vp, sz, C.POINTER(PubInputs), u32, vp, sz]
        _lib = L
    return _lib


# ---------------------------------------------------------------- element helpers
def to_bytes(values) -> bytes:
    return b"".join(int(v).to_bytes(16, "little") for v in values)


def from_bytes(b: bytes) -> list[int]:
    return [int.from_bytes(b[i:i + 16], "little") for i in range(0, len(b), 16)]


def elems_to_array(values) -> np.ndarray:
    """list of ints -> (k, 2) uint64 array (lo, hi) = 16-byte LE layout."""
    a = np.empty((len(values), 2), dtype=np.uint64)
    for i, v in enumerate(values):
        a[i, 0] = v & 0xFFFFFFFFFFFFFFFF
        a[i, 1] = v >> 64
    return a


def array_to_elems(a: np.ndarray) -> list[int]:
    a = np.ascontiguousarray(a, dtype=np.uint64).reshape(-1, 2)
    return [int(lo) | (int(hi) << 64) for lo, hi in a]


def _buf(values):
    return C.create_string_buffer(to_bytes(values), 16 * len(values))


def fop(name, a, b=None):
    out = C.create_string_buffer(16)
    if b is None:
        getattr(lib(), name)(_buf([a]), out)
    else:
        getattr(lib(), name)(_buf([a]), _buf([b]), out)
    return from_bytes(out.raw)[0]


def e2op(name, x, y=None):
    """Quadratic-extension op on (a, b) pairs (a + b*X)."""
    out = C.create_string_buffer(32)
    if y is None:
        getattr(lib(), name)(_buf(list(x)), out)
    else:
        getattr(lib(), name)(_buf(list(x)), _buf(list(y)), out)
    return tuple(from_bytes(out.raw))


def root_of_unity(log_n: int) -> int:
    out = C.create_string_buffer(16)
    lib().or_root_of_unity(log_n, out)
    return from_bytes(out.raw)[0]


def eval_coset(coeffs, size, offset):
    out = C.create_string_buffer(16 * size)
    rc = lib().or_eval_coset(_buf(coeffs), len(coeffs), size, _buf([offset]), out)
    assert rc == 0
    return from_bytes(out.raw)


def interp_coset(vals, offset):
    b = _buf(vals)
    assert lib().or_interp_coset(b, len(vals), _buf([offset])) == 0
    return from_bytes(b.raw)


def blake3(data: bytes) -> bytes:
    out = C.create_string_buffer(32)
    lib().or_blake3(data, len(data), out)
    return out.raw


def merkle_root(leaves: bytes) -> bytes:
    out = C.create_string_buffer(32)
    lib().or_merkle_root(leaves, len(leaves) // 32, out)
    return out.raw


def rescue_apply_round(state, op_code, op_value, step):
    b = _buf(state)
    lib().or_rescue_apply_round(b, op_code, op_value, step)
    return from_bytes(b.raw)


def ark(row, col):
    out = C.create_string_buffer(16)
    lib().or_rescue_ark(row, col, out)
    return from_bytes(out.raw)[0]


class OracleError(Exception):
    def __init__(self, code, message):
        super().__init__(message)
        self.code = code


def program_compile(source: str):
    cap = 16 * len(source) + 64
    codes, values = (C.c_uint8 * cap)(), (C.c_uint8 * cap)()
    n = C.c_size_t()
    h = C.create_string_buffer(32)
    msg = C.create_string_buffer(512)
    rc = lib().or_program_compile(source.encode(), codes, values, cap, C.byref(n), h, msg, 512)
    if rc:
        raise OracleError(rc, msg.value.decode())
    return list(codes[:n.value]), list(values[:n.value]), from_bytes(h.raw)


def processor_trace(codes, values, public=(), secret=(), lwe_size=5, delta=16, last_row=None):
    """Returns (trace as (28, n) uint64x2 array of ints list-of-lists, outputs list)."""
    num_ops = len(codes)
    cap = 16
    while cap <= num_ops:
        cap *= 2
    n_cap = 2 * cap
    if last_row is None:
        last_row = [1] * 28
    flat_secret = [v for ct in secret for v in ct]
    trace = C.create_string_buffer(28 * n_cap * 16)
    outputs = C.create_string_buffer(256)
    n = C.c_size_t()
    msg = C.create_string_buffer(512)
    pub_b = bytes(public)
    rc = lib().or_processor_trace(bytes(codes), bytes(values), num_ops, pub_b, len(pub_b), _buf(flat_secret),
                                  len(secret), lwe_size, delta, _buf(last_row), trace, n_cap, C.byref(n), outputs,
                                  msg, 512)
    if rc:
        raise OracleError(rc, msg.value.decode())
    arr = np.frombuffer(trace.raw[:28 * n.value * 16], dtype=np.uint64).reshape(28, n.value, 2).copy()
    return arr, from_bytes(outputs.raw)


def periodic_row(step):
    out = C.create_string_buffer(16 * 9)
    lib().or_air_periodic_row(step, out)
    return from_bytes(out.raw)


def eval_transition(cur, nxt, periodic, lwe_size=5, delta=16):
    out = C.create_string_buffer(16 * 20)
    lib().or_air_eval_transition(_buf(cur), _buf(nxt), _buf(periodic), lwe_size, delta, out)
    return from_bytes(out.raw)


def default_options(**kw) -> Options:
    o = Options(num_queries=32, blowup=8, grinding=0, field_extension=1, fri_folding=8, fri_rem_max_deg=127)
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def make_pub(program_hash, outputs, lwe_size=5, delta=16) -> PubInputs:
    p = PubInputs()
    C.memmove(p.program_hash, to_bytes(program_hash), 32)
    C.memmove(p.stack_outputs, to_bytes(list(outputs)[:16]), 256)
    p.lwe_size, p.delta = lwe_size, delta
    return p


def prove(trace: np.ndarray, pub: PubInputs, options: Options | None = None, want=()):
    """trace: (28, n, 2) uint64.  want: names of Dump fields to return as uint64 arrays."""
    rc, proof, rec, held = prove_rc(trace, pub, options, want)
    if rc != 0:
        raise OracleError(rc, f"or_prove failed with status {rc}")
    return proof, rec, held


def prove_rc(trace: np.ndarray, pub: PubInputs, options: Options | None = None, want=()):
    """prove() that returns the status instead of raising: (rc, proof, record, dumps).  A trace that
    violates the AIR still runs every stage (the stage dumps are filled) and ends with OR_ERR_DEGREE."""
    options = options or default_options()
    trace = np.ascontiguousarray(trace, dtype=np.uint64)
    n = trace.shape[1]
    N = n * options.blowup
    rec = Record()
    dump = Dump()
    sizes = {"trace_polys": 28 * n, "trace_lde": N * 28, "trace_leaves": N * 2, "composition": 8 * n,
             "comp_polys": 16 * n, "comp_lde": N * 16, "deep": N, "fri_layer1": N // options.fri_folding}
    held = {}
    for name in want:
        held[name] = np.zeros((sizes[name], 2), dtype=np.uint64)
        setattr(dump, name, held[name].ctypes.data)
    cap = 4 << 20
    buf = C.create_string_buffer(cap)
    plen = C.c_size_t(cap)
    rc = lib().or_prove(trace.ctypes.data, n, C.byref(options), C.byref(pub), buf, C.byref(plen), C.byref(rec),
                        C.byref(dump))
    return rc, (buf.raw[:plen.value] if rc == 0 else b""), rec, held


def verify(proof: bytes, pub: PubInputs, min_security: int = 95):
    msg = C.create_string_buffer(256)
    rc = lib().or_verify(proof, len(proof), C.byref(pub), min_security, msg, 256)
    return rc, msg.value.decode()
