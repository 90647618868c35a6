"""One proof with the LDE domain sharded by coset over several GPUs (zk_prove_sharded).

Rank g of `world` owns the block of LDE cosets g*Bl .. g*Bl+Bl-1 (Bl = blowup / world); block Merkle nodes,
composition coefficient slices, FRI layers 0-1 and the openings are exchanged through a communicator:

  * ShardedProver.loopback(world)       -- every rank driven from this process (one prover per rank,
                                           in-process copies); used by the tests on one GPU;
  * ShardedProver.rccl(rank, world, id) -- one process per GPU, RCCL over xGMI (the librccl the library
                                           links); the 128-byte id comes from ShardedProver.unique_id() on
                                           rank 0 and is shared out of band (bench.py: HostGroup.broadcast);
  * ShardedProver.host(rank, world, fn)  -- one process per rank, exchanges staged through host memory and
                                           a caller transport (zkvm_amd.hostgroup.HostGroup.exchange_fn():
                                           TCP; MPI or any other transport through the same C callback).
Every rank returns the same proof bytes, identical to the single-GPU prover's.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import native
from .native import Record, check, lib
from .prover import REFERENCE_OPTIONS, ProofOptions


class ShardedProver:
    def __init__(self, comm, provers, rank: int, world: int, keep=None):
        self.comm, self.provers, self.rank, self.world = comm, provers, rank, world
        self._keep = keep  # the exchange callback of a host communicator

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(lib().zk_comm_unique_id(buf), "zk_comm_unique_id")
        return buf.raw

    @classmethod
    def loopback(cls, world: int, device: int = 0, max_trace_len: int = 1 << 16) -> "ShardedProver":
        comm = C.c_void_p()
        check(lib().zk_comm_create_loopback(world, C.byref(comm)), "zk_comm_create_loopback")
        provers = []
        for _ in range(world):  # one rank's share of the LDE domain each (zk_prover_create_shard)
            p = C.c_void_p()
            check(lib().zk_prover_create_shard(device, max_trace_len, world, C.byref(p)), "zk_prover_create_shard")
            provers.append(p)
        return cls(comm, provers, 0, world)

    @classmethod
    def rccl(cls, rank: int, world: int, uid: bytes, device: int, max_trace_len: int) -> "ShardedProver":
        comm = C.c_void_p()
        check(lib().zk_comm_create_rccl(uid, rank, world, device, C.byref(comm)), "zk_comm_create_rccl")
        p = C.c_void_p()
        check(lib().zk_prover_create_shard(device, max_trace_len, world, C.byref(p)), "zk_prover_create_shard")
        return cls(comm, [p], rank, world)

    @classmethod
    def host(cls, rank: int, world: int, fn, device: int, max_trace_len: int) -> "ShardedProver":
        """One rank per process over a caller transport: fn is a native.EXCHANGE_FN (see HostGroup.exchange_fn)."""
        comm = C.c_void_p()
        check(lib().zk_comm_create_host(rank, world, fn, None, C.byref(comm)), "zk_comm_create_host")
        p = C.c_void_p()
        rc = lib().zk_prover_create_shard(device, max_trace_len, world, C.byref(p))
        if rc != native.ZK_OK:
            lib().zk_comm_destroy(comm)
            check(rc, "zk_prover_create_shard")
        return cls(comm, [p], rank, world, keep=fn)

    def upload_trace(self, trace: np.ndarray) -> int:
        """Copy the trace into every local prover's device trace buffer (then prove(None, n=...))."""
        from .prover import _hip
        trace = np.ascontiguousarray(trace, dtype=np.uint64)
        for p in self.provers:
            d = C.c_void_p()
            check(lib().zk_prover_trace_buffer(p, C.byref(d)), "zk_prover_trace_buffer")
            rc = _hip().hipMemcpy(d, trace.ctypes.data_as(C.c_void_p), trace.nbytes, 1)
            if rc != 0:
                raise native.ZkError(native.ZK_ERR_DEVICE, f"hipMemcpy failed ({rc})")
        return trace.shape[1]

    def prove(self, trace, pub, options: ProofOptions = REFERENCE_OPTIONS, record: bool = False, n: int = 0):
        """trace: (28, n, 2) uint64 host array, or None with n= to prove the uploaded trace."""
        if trace is not None:
            trace = np.ascontiguousarray(trace, dtype=np.uint64)
            n = trace.shape[1]
        opt = options.to_c()
        if getattr(self, "_proof_buf", None) is None:  # reused across proofs (see GpuProver.prove_device)
            self._proof_buf = C.create_string_buffer(4 << 20)
        buf = self._proof_buf
        plen = C.c_size_t(len(buf))
        rec = Record() if record else None
        arr = (C.c_void_p * len(self.provers))(*[p.value for p in self.provers])
        rc = lib().zk_prove_sharded(self.comm, arr, len(self.provers),
                                    trace.ctypes.data if trace is not None else None, n, C.byref(opt),
                                    C.byref(pub), buf, C.byref(plen), C.byref(rec) if rec is not None else None)
        check(rc, "zk_prove_sharded")
        return C.string_at(buf, plen.value), rec

    def prove_program(self, prog, inputs, last_row, options: ProofOptions = REFERENCE_OPTIONS):
        """vm::prove sharded (zk_vm_prove_sharded): every local rank writes the trace of `prog` on `inputs`
        (Program.encode_inputs) into its own HBM, then one proof over the ranks.  last_row is required (the same
        on every rank).  Returns (program hash, outputs, proof)."""
        from .prover import bytes_elems, elems_bytes
        opt = options.to_c()
        if getattr(self, "_proof_buf", None) is None:
            self._proof_buf = C.create_string_buffer(4 << 20)
        buf = self._proof_buf
        plen = C.c_size_t(len(buf))
        outputs = C.create_string_buffer(256)
        h = C.create_string_buffer(32)
        arr = (C.c_void_p * len(self.provers))(*[p.value for p in self.provers])
        rc = lib().zk_vm_prove_sharded(self.comm, arr, len(self.provers), prog.handle, *inputs, elems_bytes(last_row),
                                       C.byref(opt), buf, C.byref(plen), outputs, h)
        check(rc, "zk_vm_prove_sharded")
        return bytes_elems(h.raw), bytes_elems(outputs.raw), C.string_at(buf, plen.value)

    def stage_times(self) -> dict:
        names = (C.c_char_p * 32)()
        ms = (C.c_float * 32)()
        cnt = C.c_int(0)
        lib().zk_prover_stage_times(self.provers[0], names, ms, 32, C.byref(cnt))
        return {names[i].decode(): ms[i] for i in range(cnt.value)}

    def exchange_stats(self, exposed: bool = False) -> dict:
        """{collective: (ms, bytes received from the other ranks, calls)} of the last proof on local rank 0
        (zk_prover_exchange_stats): events around each collective on the stream it ran on, so the time includes waiting
        for peers.  exposed=True appends the exposed ms (how long the compute stream waited for it) to each tuple."""
        names = (C.c_char_p * 32)()
        ms = (C.c_float * 32)()
        ex = (C.c_float * 32)()
        by = (C.c_double * 32)()
        calls = (C.c_int * 32)()
        cnt = C.c_int(0)
        check(lib().zk_prover_exchange_stats_ex(self.provers[0], names, ms, ex, by, calls, 32, C.byref(cnt)))
        k = min(cnt.value, 32)
        if exposed:
            return {names[i].decode(): (ms[i], by[i], calls[i], ex[i]) for i in range(k)}
        return {names[i].decode(): (ms[i], by[i], calls[i]) for i in range(k)}

    def set_measure(self, on: bool):
        """zk_comm_set_measure (loopback only): serialise every rank's compute and the exchange copies on one stream,
        so the schedule's segments are the ranks' compute alone (tools/shard_model.py); the proof bytes are unchanged."""
        check(lib().zk_comm_set_measure(self.comm, 1 if on else 0))

    def set_trace_split(self, replicated: int = -1):
        """zk_comm_set_trace_split: trace columns every rank interpolates itself when the trace is in every rank's HBM
        (-1: the library's choice per world size); the proof bytes do not depend on it."""
        check(lib().zk_comm_set_trace_split(self.comm, int(replicated)))

    def schedule(self) -> dict:
        """The last proof's schedule on local rank 0 (zk_prover_shard_schedule): exchange starts / waits in issue
        order and the measured compute segments between them."""
        import json
        need = C.c_size_t(0)
        lib().zk_prover_shard_schedule(self.provers[0], None, 0, C.byref(need))
        buf = C.create_string_buffer(need.value)
        check(lib().zk_prover_shard_schedule(self.provers[0], buf, need.value, C.byref(need)))
        return json.loads(buf.value.decode())

    def close(self):
        for p in self.provers:
            lib().zk_prover_destroy(p)
        self.provers = []
        if self.comm:
            lib().zk_comm_destroy(self.comm)
            self.comm = None
