"""Host-side mirror of the reference's prover surface, driving the gfx950 library.

Reference interface mirrored here (same names, argument meaning and error behaviour):
  * ProofOptions::new(num_queries, blowup, grinding, field_extension, fri_folding, rem_max_degree)
    (winterfell 0.9; hard-coded as (32, 8, 0, None, 8, 127) at vm/src/lib.rs:20)
  * ExecutionProver::new(options, program_hash, stack_outputs, server_key)  prover/src/lib.rs:25-37
  * Prover::prove(trace) -> Proof                                           prover/src/lib.rs:40-77
  * vm::prove(program, inputs) -> (hash, outputs, proof)                     vm/src/lib.rs:13-29
The trace is the 28-column matrix of vm/src/processor/mod.rs:71-95 as a (28, n, 2) uint64 array
(low, high halves of each canonical f128 value) or any buffer with that byte layout.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import native
from .native import Dump, Options, PubInputs, Record, ZkError, check, lib

P = 2**128 - 45 * 2**40 + 1
FIELD_EXTENSION_NONE = 1
FIELD_EXTENSION_QUADRATIC = 2


@dataclass(frozen=True)
class ProofOptions:
    num_queries: int = 32
    blowup_factor: int = 8
    grinding_factor: int = 0
    field_extension: int = FIELD_EXTENSION_NONE
    fri_folding_factor: int = 8
    fri_remainder_max_degree: int = 127

    def to_c(self) -> Options:
        return Options(self.num_queries, self.blowup_factor, self.grinding_factor, self.field_extension,
                       self.fri_folding_factor, self.fri_remainder_max_degree)


REFERENCE_OPTIONS = ProofOptions()  # vm/src/lib.rs:20


def elems_bytes(values) -> bytes:
    return b"".join(int(v).to_bytes(16, "little") for v in values)


def bytes_elems(b: bytes) -> list[int]:
    return [int.from_bytes(b[i:i + 16], "little") for i in range(0, len(b), 16)]


def make_pub_inputs(program_hash, stack_outputs, lwe_size: int, delta: int) -> PubInputs:
    p = PubInputs()
    C.memmove(p.program_hash, elems_bytes(program_hash), 32)
    C.memmove(p.stack_outputs, elems_bytes(list(stack_outputs)[:16]), 256)
    p.lwe_size, p.delta = lwe_size, delta
    return p


class GpuProver:
    """One GPU's device memory and stream (zk_prover)."""

    def __init__(self, device: int = 0, max_trace_len: int = 1 << 16, max_blowup: int = 8, pooled: bool = False):
        """pooled: take the prover from the process-wide pool (zk_prover_acquire) and hand it back on close
        (zk_prover_release) instead of creating and freeing it -- the per-call construction of the reference
        (ExecutionProver::new in vm::prove) at the cost of a pool lookup."""
        h = C.c_void_p()
        if pooled:
            check(lib().zk_prover_acquire(device, max_trace_len, max_blowup, C.byref(h)), "zk_prover_acquire")
        else:
            check(lib().zk_prover_create(device, max_trace_len, max_blowup, C.byref(h)), "zk_prover_create")
        self.handle = h
        self.max_trace_len = max_trace_len
        self.device = device
        self.pooled = pooled

    def close(self):
        if self.handle:
            (lib().zk_prover_release if self.pooled else lib().zk_prover_destroy)(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def trace_buffer(self) -> int:
        p = C.c_void_p()
        check(lib().zk_prover_trace_buffer(self.handle, C.byref(p)), "zk_prover_trace_buffer")
        return p.value

    def prove_device(self, d_trace: int, n: int, pub: PubInputs, options: ProofOptions = REFERENCE_OPTIONS,
                     record: bool = False, dump=(), allow_degree_error=False):
        """zk_prove_device: the trace is already in this prover's HBM (upload_trace)."""
        return self._prove(lambda *a: lib().zk_prove_device(self.handle, d_trace, n, *a), n, pub, options, record,
                           dump, allow_degree_error)

    def prove_host(self, trace: np.ndarray, pub: PubInputs, options: ProofOptions = REFERENCE_OPTIONS,
                   record: bool = False, dump=(), allow_degree_error=False):
        """zk_prove_columns_ex: the trace is a (28, n, 2) uint64 host array (pinned -- HostTrace -- or
        pageable); the library uploads it column group by column group, overlapped with the interpolation."""
        trace = np.ascontiguousarray(trace, dtype=np.uint64)
        assert trace.ndim == 3 and trace.shape[0] == 28 and trace.shape[2] == 2
        n = trace.shape[1]
        if getattr(self, "_cols", None) is None:
            self._cols = (C.c_void_p * 28)()
        cols = self._cols
        base, stride = trace.ctypes.data, trace.strides[0]
        for c in range(28):
            cols[c] = base + c * stride
        return self._prove(lambda *a: lib().zk_prove_columns_ex(self.handle, cols, n, *a), n, pub, options, record,
                           dump, allow_degree_error)

    def _prove(self, call, n, pub, options, record, dump, allow_degree_error):
        opt = options.to_c()
        # one proof buffer per prover, reused across proofs (a fresh 4 MiB ctypes buffer per call was
        # ~0.15 ms of zero-fill and page faults between two proofs); only plen bytes are copied out
        if getattr(self, "_proof_buf", None) is None:
            self._proof_buf = C.create_string_buffer(4 << 20)
        buf = self._proof_buf
        plen = C.c_size_t(len(buf))
        rec = Record() if record else None
        held = {}
        dmp = None
        if dump:
            dmp = Dump()
            N = n * options.blowup_factor
            sizes = {"trace_polys": 28 * n, "trace_lde": N * 28, "trace_leaves": N * 2, "composition": 8 * n,
                     "comp_polys": 16 * n, "comp_lde": N * 16, "deep": N,
                     "fri_layer1": max(1, N // options.fri_folding_factor)}
            for name in dump:
                held[name] = np.zeros((sizes[name], 2), dtype=np.uint64)
                setattr(dmp, name, held[name].ctypes.data)
        rc = call(C.byref(opt), C.byref(pub), buf, C.byref(plen), C.byref(rec) if rec is not None else None,
                  C.byref(dmp) if dmp is not None else None)
        if not (rc == 0 or (allow_degree_error and rc == native.ZK_ERR_DEGREE)):
            check(rc, "prove")
        return C.string_at(buf, plen.value), rec, held, rc

    def upload_trace(self, trace: np.ndarray) -> tuple[int, int]:
        """Copy a (28, n, 2) uint64 host trace into this prover's device trace buffer."""
        import ctypes
        trace = np.ascontiguousarray(trace, dtype=np.uint64)
        assert trace.shape[0] == 28 and trace.shape[2] == 2
        n = trace.shape[1]
        if n > self.max_trace_len:
            raise ZkError(native.ZK_ERR_INVALID_ARG, "trace longer than max_trace_len")
        d = self.trace_buffer()
        hip = _hip()
        rc = hip.hipMemcpy(ctypes.c_void_p(d), trace.ctypes.data_as(ctypes.c_void_p), trace.nbytes, 1)
        if rc != 0:
            raise ZkError(native.ZK_ERR_DEVICE, f"hipMemcpy failed ({rc})")
        return d, n

    def prove(self, trace: np.ndarray, pub: PubInputs, options: ProofOptions = REFERENCE_OPTIONS, **kw):
        """Prover::prove(trace) with a host-resident trace (the reference's call shape, vm/src/lib.rs:26)."""
        if trace.shape[1] > self.max_trace_len:
            raise ZkError(native.ZK_ERR_INVALID_ARG, "trace longer than max_trace_len")
        return self.prove_host(trace, pub, options, **kw)

    def stage_times(self) -> dict:
        names = (C.c_char_p * 32)()
        ms = (C.c_float * 32)()
        cnt = C.c_int(0)
        check(lib().zk_prover_stage_times(self.handle, names, ms, 32, C.byref(cnt)))
        return {names[i].decode(): ms[i] for i in range(min(cnt.value, 32))}

    def upload_stats(self) -> dict:
        """The last host-column proof's trace upload (zk_prover_upload_stats): bytes, and the columns taken as sparse,
        uploaded packed as 8- / 32-bit integers, or derived from the AIR (the clock, zk_prover_upload_derived)."""
        b = C.c_uint64(0)
        sp, n8, n32 = C.c_uint32(0), C.c_uint32(0), C.c_uint32(0)
        check(lib().zk_prover_upload_stats(self.handle, C.byref(b), C.byref(sp), C.byref(n8), C.byref(n32)))
        dv = C.c_uint32(0)
        check(lib().zk_prover_upload_derived(self.handle, C.byref(dv)))
        cols = lambda m: [c for c in range(28) if (m >> c) & 1]  # noqa: E731
        return {"bytes": b.value, "sparse": cols(sp.value), "narrow8": cols(n8.value), "narrow32": cols(n32.value),
                "derived": cols(dv.value)}

    UPLOAD_SCHEDULES = {"auto": 0, "throughput": 1, "latency": 2}

    def proof_info(self) -> dict:
        """zk_prover_proof_info: the upload schedule the last host-column proof ran ("throughput" / "latency", None after
        a device-trace proof), the proofs voided by a refuted column hint and redone (cumulative), the (n, program) hint
        sets held, and the sparse / derived columns the last proof took from its hints."""
        from .native import ProofInfo
        info = ProofInfo()
        check(lib().zk_prover_proof_info(self.handle, C.byref(info)))
        cols = lambda m: [c for c in range(28) if (m >> c) & 1]  # noqa: E731
        return {"schedule": {1: "throughput", 2: "latency"}.get(info.schedule), "hint_redos": info.hint_redos,
                "hint_sets": info.hint_sets, "hinted_sparse": cols(info.hinted_sparse), "derived": cols(info.derived)}

    def set_upload_schedule(self, schedule: str):
        """zk_prover_set_upload_schedule: "auto" (latency when no other proof is in flight on the device), "throughput"
        or "latency" -- how a host-resident trace goes up; the proof bytes are the same."""
        check(lib().zk_prover_set_upload_schedule(self.handle, self.UPLOAD_SCHEDULES[schedule]))

    def profile(self, on: bool):
        check(lib().zk_prover_profile(self.handle, 1 if on else 0))
        check(lib().zk_prover_kernel_stats(self.handle, None, None, None, None, 0, None))  # reset

    def kernel_stats(self) -> dict:
        """{kernel: (total_ms, launches, algorithmic_bytes)} since the last profile(True)."""
        names = (C.c_char_p * 64)()
        ms = (C.c_float * 64)()
        nl = (C.c_int * 64)()
        by = (C.c_double * 64)()
        cnt = C.c_int(0)
        check(lib().zk_prover_kernel_stats(self.handle, names, ms, nl, by, 64, C.byref(cnt)))
        return {names[i].decode(): (ms[i], nl[i], by[i]) for i in range(min(cnt.value, 64))}

    def kernel_ops(self) -> dict:
        """{kernel: (f128 multiplies, f128 additions/subtractions)} for the kernels whose operation
        count the library models (the NTT passes), accumulated like kernel_stats."""
        names = (C.c_char_p * 64)()
        ms = (C.c_float * 64)()
        nl = (C.c_int * 64)()
        by = (C.c_double * 64)()
        mu = (C.c_double * 64)()
        ad = (C.c_double * 64)()
        cnt = C.c_int(0)
        check(lib().zk_prover_kernel_stats(self.handle, names, ms, nl, by, 64, C.byref(cnt)))
        check(lib().zk_prover_kernel_ops(self.handle, mu, ad, 64, C.byref(cnt)))
        return {names[i].decode(): (mu[i], ad[i]) for i in range(min(cnt.value, 64)) if mu[i] or ad[i]}


class _PinnedBlock:
    """Owner of one zk_host_alloc block.  numpy arrays over it keep it as their base (__array_interface__), so
    the block is freed only when the last array that views it is gone."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(lib().zk_host_alloc(nbytes, C.byref(p)), "zk_host_alloc")
        self.ptr = p.value
        self.__array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (self.ptr, False), "version": 3}

    def __del__(self):
        try:
            if self.ptr:
                lib().zk_host_free(C.c_void_p(self.ptr))
                self.ptr = None
        except Exception:
            pass


class HostTrace:
    """A (28, n, 2) uint64 trace array in page-locked host memory (zk_host_alloc): the VM writes into it
    (vm_trace(..., out=...)) and zk_prove DMAs it at the link rate.  close() (or a with-block) drops this
    object's reference; the memory goes back once no array returned from it (trace(..., out=...)) is alive."""

    def __init__(self, n: int):
        self.n = n
        self.array = np.asarray(_PinnedBlock(28 * n * 16)).view(np.uint64).reshape(28, n, 2)

    @property
    def ptr(self):
        return None if self.array is None else self.array.ctypes.data

    def close(self):
        self.array = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_hip_lib = None


def _hip():
    global _hip_lib
    if _hip_lib is None:
        _hip_lib = native.hip_runtime()  # the runtime the library runs on, never a second copy
    return _hip_lib


class ExecutionProver:
    """prover/src/lib.rs:17-77 -- `ExecutionProver::new(options, program_hash, stack_outputs, server_key)`
    then `.prove(trace)`.  Panics in the reference (`prove(...).unwrap()`, vm/src/lib.rs:26) become
    ZkError here."""

    def __init__(self, options: ProofOptions, program_hash, stack_outputs, server_key, gpu: GpuProver | None = None):
        self.options = options
        self.program_hash = list(program_hash)
        self.stack_outputs = list(stack_outputs)
        self.server_key = server_key
        self._gpu = gpu

    def get_pub_inputs(self) -> PubInputs:
        return make_pub_inputs(self.program_hash, self.stack_outputs, self.server_key.lwe_size(),
                               self.server_key.parameters.delta)

    def prove(self, trace: np.ndarray) -> bytes:
        n = trace.shape[1]
        gpu = self._gpu or GpuProver(0, max(n, 16), max(8, self.options.blowup_factor))
        proof, _, _, _ = gpu.prove(trace, self.get_pub_inputs(), self.options)
        return proof


# ------------------------------------------------------------------ VM harness (vm::prove)
def verify(proof: bytes, pub: PubInputs, min_security: int = 95) -> tuple[int, str]:
    """winterfell::verify (vm/src/lib.rs:93-98) for this library's proofs, on the host: (status, reason)."""
    msg = C.create_string_buffer(256)
    rc = lib().zk_verify(proof, len(proof), C.byref(pub), min_security, msg, 256)
    return rc, msg.value.decode()


def vm_trace(source: str, public, secret, server_key, last_row, out=None):
    """Processor::run + trace (vm/src/processor/mod.rs:61-95) via the native VM.
    Returns (trace (28, n, 2) uint64, outputs[16], program_hash[2]).  out: an optional HostTrace (or a
    C-contiguous (28, n, 2) uint64 array) of exactly the trace's length to write the trace into."""
    L = server_key.lwe_size()
    sec = elems_bytes([v for ct in secret for v in ct])
    nops_hint = 16 * len(source) + 64
    cap = 16
    while cap <= nops_hint:
        cap *= 2
    cap *= 2
    n = C.c_size_t(0)
    outputs = C.create_string_buffer(256)
    h = C.create_string_buffer(32)
    # first call: size query
    rc = lib().zk_vm_trace(source.encode(), bytes(public), len(public), sec, len(secret), L,
                           server_key.parameters.delta, elems_bytes(last_row), None, 0, C.byref(n), outputs, h)
    if rc not in (0, native.ZK_ERR_BUFFER_TOO_SMALL):
        raise ZkError(rc, lib().zk_vm_last_error().decode())
    if out is None:
        trace = np.zeros((28, n.value, 2), dtype=np.uint64)
    else:
        trace = out.array if isinstance(out, HostTrace) else out
        if trace.shape != (28, n.value, 2) or trace.dtype != np.uint64 or not trace.flags.c_contiguous:
            raise ZkError(native.ZK_ERR_INVALID_ARG, f"out must be a contiguous (28, {n.value}, 2) uint64 array")
    rc = lib().zk_vm_trace(source.encode(), bytes(public), len(public), sec, len(secret), L,
                           server_key.parameters.delta, elems_bytes(last_row), trace.ctypes.data, n.value,
                           C.byref(n), outputs, h)
    if rc:
        raise ZkError(rc, lib().zk_vm_last_error().decode())
    return trace, bytes_elems(outputs.raw), bytes_elems(h.raw)


class Program:
    """Program::compile (vm/src/program/mod.rs:37-131) through zk_program_compile: parse, pad, hash.  The handle
    keeps the chiplet's per-step sponge states (a function of the code alone), so trace() -- Processor::run +
    trace on given inputs (vm/src/processor/mod.rs:61-95) -- is the stack machine plus threaded row writes."""

    def __init__(self, source: str):
        h = C.c_void_p()
        hb = C.create_string_buffer(32)
        n = C.c_size_t(0)
        rc = lib().zk_program_compile(source.encode(), C.byref(h), hb, C.byref(n))
        if rc:
            raise ZkError(rc, lib().zk_vm_last_error().decode())
        self.handle = h
        self.hash = bytes_elems(hb.raw)
        self.trace_len = n.value

    def trace(self, public, secret, server_key, last_row, out=None):
        """Returns (trace (28, n, 2) uint64, outputs[16]); out: an optional HostTrace / array of length n."""
        n = self.trace_len
        if out is None:
            trace = np.zeros((28, n, 2), dtype=np.uint64)
        else:
            trace = out.array if isinstance(out, HostTrace) else out
            if trace.shape != (28, n, 2) or trace.dtype != np.uint64 or not trace.flags.c_contiguous:
                raise ZkError(native.ZK_ERR_INVALID_ARG, f"out must be a contiguous (28, {n}, 2) uint64 array")
        sec = elems_bytes([v for ct in secret for v in ct])
        outputs = C.create_string_buffer(256)
        nn = C.c_size_t(0)
        rc = lib().zk_program_trace(self.handle, bytes(public), len(public), sec, len(secret), server_key.lwe_size(),
                                    server_key.parameters.delta, elems_bytes(last_row), trace.ctypes.data, n,
                                    C.byref(nn), outputs)
        if rc:
            raise ZkError(rc, lib().zk_vm_last_error().decode())
        return trace, bytes_elems(outputs.raw)

    @staticmethod
    def encode_inputs(public, secret, server_key):
        """ProgramInputs in the C ABI's form (public u8 bytes, secret ciphertexts as 16-byte elements, lwe_size,
        delta): encode once, run many times."""
        sec = elems_bytes([v for ct in secret for v in ct])
        return (bytes(public), len(public), sec, len(secret), server_key.lwe_size(), server_key.parameters.delta)

    def trace_device(self, gpu: "GpuProver", inputs, last_row=None):
        """Processor::run + trace written by the GPU into gpu's trace buffer (zk_vm_trace_device); inputs from
        encode_inputs.  Returns (device pointer, n, outputs[16]).  last_row None: drawn at random, as
        Processor::trace does."""
        n = C.c_size_t(0)
        outputs = C.create_string_buffer(256)
        rc = lib().zk_vm_trace_device(gpu.handle, self.handle, *inputs,
                                      elems_bytes(last_row) if last_row is not None else None, C.byref(n), outputs)
        if rc:
            check(rc, "zk_vm_trace_device")
        return gpu.trace_buffer(), n.value, bytes_elems(outputs.raw)

    def prove_device(self, gpu: "GpuProver", inputs, last_row=None, options: ProofOptions = None):
        """vm::prove (vm/src/lib.rs:13-29) with the trace generated on the GPU (zk_vm_prove); inputs from
        encode_inputs.  Returns (hash, outputs, proof)."""
        opt = (options or REFERENCE_OPTIONS).to_c()
        if getattr(gpu, "_proof_buf", None) is None:
            gpu._proof_buf = C.create_string_buffer(4 << 20)
        buf = gpu._proof_buf
        plen = C.c_size_t(len(buf))
        outputs = C.create_string_buffer(256)
        h = C.create_string_buffer(32)
        rc = lib().zk_vm_prove(gpu.handle, self.handle, *inputs,
                               elems_bytes(last_row) if last_row is not None else None, C.byref(opt), buf,
                               C.byref(plen), outputs, h)
        if rc:
            check(rc, "zk_vm_prove")
        return bytes_elems(h.raw), bytes_elems(outputs.raw), C.string_at(buf, plen.value)

    def stack_states(self, public, secret, server_key, stride: int, count: int):
        """The host stack pass behind the device generator (diagnostics): (states as a (count, 17, 2) uint64 array --
        16 registers top first, then [depth | ta << 32, tb] -- and outputs[16]); state c is what row c*stride - 1
        shows."""
        out = np.zeros((count, 17, 2), dtype=np.uint64)
        outputs = C.create_string_buffer(256)
        rc = lib().zk_diag_vm_states(self.handle, *self.encode_inputs(public, secret, server_key), stride, count,
                                     out.ctypes.data, outputs)
        if rc:
            raise ZkError(rc, lib().zk_vm_last_error().decode())
        return out, bytes_elems(outputs.raw)

    def close(self):
        if self.handle:
            lib().zk_program_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def prove(source: str, public, secret, server_key, last_row, options: ProofOptions = REFERENCE_OPTIONS,
          gpu: GpuProver | None = None):
    """vm::prove (vm/src/lib.rs:13-29): run -> output -> trace -> options -> hash -> prove."""
    trace, outputs, program_hash = vm_trace(source, public, secret, server_key, last_row)
    prover = ExecutionProver(options, program_hash, outputs, server_key, gpu)
    return program_hash, outputs, prover.prove(trace)
