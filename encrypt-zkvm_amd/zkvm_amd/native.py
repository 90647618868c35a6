"""ctypes binding of libzkvm_gpu.so (include/zkvm_gpu.h).

The product path: every prove goes through this library's HIP kernels.  There is no CPU
fallback -- if the library is missing, loading fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent
# ZKVM_GPU_LIB selects an alternative in-tree build (A/B experiments); default lib/libzkvm_gpu.so
LIB_PATH = Path(os.environ.get("ZKVM_GPU_LIB", PKG_ROOT / "lib" / "libzkvm_gpu.so"))

ZK_OK = 0
ZK_ERR_INVALID_ARG = -1
ZK_ERR_BUFFER_TOO_SMALL = -2
ZK_ERR_DEVICE = -3
ZK_ERR_OUT_OF_MEMORY = -4
ZK_ERR_PROGRAM = -10
ZK_ERR_STACK = -11
ZK_ERR_CHIPLETS = -12
ZK_ERR_DEGREE = -20
ZK_ERR_VERIFY = -30

MAX_COLS, MAX_TCONS, MAX_ASSERTS, MAX_CCOLS, MAX_FRI, MAX_REM, MAX_Q = 32, 32, 32, 16, 16, 256, 255

# every symbol include/zkvm_gpu.h declares (checked by tests/test_native_abi.py)
EXPORTED = (
    "zk_last_error", "zk_device_count", "zk_runtime_versions", "zk_device_pci_bus_id", "zk_device_synchronize",
    "zk_prover_create", "zk_prover_create_shard", "zk_prover_destroy",
    "zk_prover_acquire", "zk_prover_release", "zk_prover_pool_trim", "zk_prover_trace_buffer",
    "zk_prove", "zk_prove_columns", "zk_prove_columns_ex", "zk_host_alloc", "zk_host_free", "zk_host_register",
    "zk_host_unregister", "zk_prove_device", "zk_lde_new", "zk_lde_read_frame", "zk_lde_query", "zk_lde_free",
    "zk_eval_constraints", "zk_commit_composition", "zk_comp_query", "zk_comp_free", "zk_prover_stage_times", "zk_prover_profile", "zk_prover_kernel_stats", "zk_prover_kernel_ops", "zk_prover_exchange_stats", "zk_prover_exchange_stats_ex", "zk_prover_shard_schedule", "zk_prover_upload_stats", "zk_prover_upload_derived", "zk_prover_set_upload_schedule", "zk_prover_proof_info", "zk_vm_trace",
    "zk_verify", "zk_comm_create_loopback", "zk_comm_unique_id", "zk_comm_create_rccl", "zk_comm_create_host", "zk_comm_destroy", "zk_comm_set_measure", "zk_comm_set_trace_split", "zk_prove_sharded",
    "zk_program_compile", "zk_program_trace", "zk_program_free", "zk_vm_last_error", "zk_vm_trace_device",
    "zk_vm_prove",
    "zk_vm_prove_sharded",
)


# zk_exchange_fn (include/zkvm_gpu.h): int fn(void *ctx, int op, const void *send, void *recv, size_t bytes)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t)
XCHG_ALL_TO_ALL, XCHG_ALL_GATHER = 0, 1


class ZkError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"[{code}] {message}")
        self.code = code


class Options(C.Structure):
    _fields_ = [(f, C.c_uint32) for f in
                ("num_queries", "blowup", "grinding", "field_extension", "fri_folding", "fri_rem_max_deg")]


class PubInputs(C.Structure):
    _fields_ = [("program_hash", C.c_uint8 * 32), ("stack_outputs", C.c_uint8 * 256),
                ("lwe_size", C.c_uint32), ("delta", C.c_uint32)]


class ProofInfo(C.Structure):
    """zk_proof_info (include/zkvm_gpu.h): what the last proof on a prover did."""
    _fields_ = [("schedule", C.c_int32), ("hint_redos", C.c_uint32), ("hint_sets", C.c_uint32),
                ("hinted_sparse", C.c_uint32), ("derived", C.c_uint32), ("_pad", C.c_uint32)]


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


_lib = None
_runtime = None


def mapped_files(prefix: str) -> list:
    """Distinct files (resolved paths) mapped into this process whose name starts with `prefix`."""
    found = set()
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split(None, 5)
            if len(parts) == 6 and os.path.basename(parts[5].strip()).startswith(prefix):
                found.add(os.path.realpath(parts[5].strip()))
    return sorted(found)


class _RefuseSecondRuntime:
    """sys.meta_path guard installed once the library has mapped the HIP runtime it links (/opt/rocm): importing
    torch afterwards would map torch's bundled libamdhip64 as a SECOND runtime (torch asks for the soname
    libamdhip64.so, which the loaded libamdhip64.so.7 does not satisfy).  A process that needs both must import
    torch first; the library then shares torch's copy (one runtime, recorded by runtime_info())."""

    def find_spec(self, name, path=None, target=None):
        if name == "torch" or name.startswith("torch."):
            raise ImportError(
                f"zkvm_amd: {LIB_PATH.name} has already mapped {runtime_info()['hip_runtime']}; importing torch now "
                f"would load torch's own HIP runtime as a second one -- import torch before the first native.lib() "
                f"call, or keep GPU work torch-free")
        return None


def runtime_info() -> dict:
    """The HIP runtime and RCCL this process's library runs on: the mapped files and their versions."""
    global _runtime
    if _runtime is None:
        L = lib()
        hv, rv = C.c_int(0), C.c_int(0)
        rc = L.zk_runtime_versions(C.byref(hv), C.byref(rv))
        hips, rccls = mapped_files("libamdhip64.so"), mapped_files("librccl.so")
        _runtime = {"hip_runtime": hips[0] if len(hips) == 1 else hips, "rccl": rccls[0] if len(rccls) == 1 else rccls,
                    "hip_runtime_version": hv.value if rc == ZK_OK else None,
                    "rccl_version": rv.value if rc == ZK_OK else None,
                    "torch_loaded_first": "torch" in __import__("sys").modules}
    return dict(_runtime)


def lib():
    global _lib
    if _lib is None:
        import sys
        if not LIB_PATH.exists():
            raise ZkError(ZK_ERR_DEVICE, f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C encrypt-zkvm_amd)")
        L = C.CDLL(str(LIB_PATH))
        hips = mapped_files("libamdhip64.so")
        if len(hips) != 1:
            raise ZkError(ZK_ERR_DEVICE, f"{len(hips)} HIP runtimes mapped into this process ({hips}): exactly one "
                                         f"must serve {LIB_PATH.name}")
        if "torch" not in sys.modules and not any(isinstance(f, _RefuseSecondRuntime) for f in sys.meta_path):
            sys.meta_path.insert(0, _RefuseSecondRuntime())
        vp, sz, u32, i32 = C.c_void_p, C.c_size_t, C.c_uint32, C.c_int
        L.zk_last_error.restype = C.c_char_p
        L.zk_device_count.argtypes = [C.POINTER(i32)]
        L.zk_runtime_versions.argtypes = [C.POINTER(i32), C.POINTER(i32)]
        L.zk_device_pci_bus_id.argtypes = [i32, C.c_char_p, i32]
        L.zk_device_synchronize.argtypes = [i32]
        L.zk_prover_create.argtypes = [i32, sz, u32, C.POINTER(vp)]
        L.zk_prover_create_shard.argtypes = [i32, sz, i32, C.POINTER(vp)]
        L.zk_prover_destroy.argtypes = [vp]
        L.zk_prover_destroy.restype = None
        L.zk_prover_acquire.argtypes = [i32, sz, u32, C.POINTER(vp)]
        L.zk_prover_release.argtypes = [vp]
        L.zk_prover_release.restype = None
        L.zk_prover_pool_trim.argtypes = [i32]
        L.zk_prover_trace_buffer.argtypes = [vp, C.POINTER(vp)]
        L.zk_prove.argtypes = [vp, vp, sz, C.POINTER(Options), C.POINTER(PubInputs), vp, C.POINTER(sz)]
        L.zk_prove_columns.argtypes = [vp, C.POINTER(vp), sz, C.POINTER(Options), C.POINTER(PubInputs), vp,
                                       C.POINTER(sz)]
        L.zk_prove_columns_ex.argtypes = [vp, C.POINTER(vp), sz, C.POINTER(Options), C.POINTER(PubInputs), vp,
                                          C.POINTER(sz), C.POINTER(Record), C.POINTER(Dump)]
        L.zk_host_alloc.argtypes = [sz, C.POINTER(vp)]
        L.zk_host_free.argtypes = [vp]
        L.zk_host_free.restype = None
        L.zk_host_register.argtypes = [vp, sz]
        L.zk_host_unregister.argtypes = [vp]
        L.zk_prove_device.argtypes = [vp, vp, sz, C.POINTER(Options), C.POINTER(PubInputs), vp, C.POINTER(sz),
                                      C.POINTER(Record), C.POINTER(Dump)]
        L.zk_lde_new.argtypes = [vp, vp, sz, sz, u32, C.POINTER(vp), vp]
        L.zk_lde_read_frame.argtypes = [vp, sz, vp, vp]
        L.zk_lde_query.argtypes = [vp, vp, sz, vp, vp, C.POINTER(sz)]
        L.zk_lde_free.argtypes = [vp]
        L.zk_lde_free.restype = None
        L.zk_eval_constraints.argtypes = [vp, C.POINTER(PubInputs), vp, vp, vp]
        L.zk_commit_composition.argtypes = [vp, vp, u32, C.POINTER(vp), vp, vp]
        L.zk_comp_query.argtypes = [vp, vp, sz, vp, vp, C.POINTER(sz)]
        L.zk_comp_free.argtypes = [vp]
        L.zk_comp_free.restype = None
        L.zk_prover_stage_times.argtypes = [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_float), i32, C.POINTER(i32)]
        L.zk_prover_profile.argtypes = [vp, i32]
        L.zk_prover_set_upload_schedule.argtypes = [vp, i32]
        L.zk_prover_proof_info.argtypes = [vp, C.POINTER(ProofInfo)]
        L.zk_prover_kernel_stats.argtypes = [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.POINTER(i32),
                                             C.POINTER(C.c_double), i32, C.POINTER(i32)]
        L.zk_prover_kernel_ops.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), i32, C.POINTER(i32)]
        L.zk_prover_upload_stats.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)]
        L.zk_prover_upload_derived.argtypes = [vp, C.POINTER(u32)]
        L.zk_prover_exchange_stats.argtypes = [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.POINTER(C.c_double),
                                               C.POINTER(i32), i32, C.POINTER(i32)]
        L.zk_verify.argtypes = [vp, sz, C.POINTER(PubInputs), u32, C.c_char_p, sz]
        L.zk_comm_create_loopback.argtypes = [i32, C.POINTER(vp)]
        L.zk_comm_unique_id.argtypes = [vp]
        L.zk_comm_create_rccl.argtypes = [vp, i32, i32, i32, C.POINTER(vp)]
        L.zk_comm_create_host.argtypes = [i32, i32, EXCHANGE_FN, vp, C.POINTER(vp)]
        L.zk_comm_destroy.argtypes = [vp]
        L.zk_comm_destroy.restype = None
        L.zk_comm_set_measure.argtypes = [vp, i32]
        L.zk_comm_set_trace_split.argtypes = [vp, i32]
        L.zk_prover_exchange_stats_ex.argtypes = [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                                  C.POINTER(C.c_double), C.POINTER(i32), i32, C.POINTER(i32)]
        L.zk_prover_shard_schedule.argtypes = [vp, C.c_char_p, sz, C.POINTER(sz)]
        L.zk_prove_sharded.argtypes = [vp, C.POINTER(vp), i32, vp, sz, C.POINTER(Options), C.POINTER(PubInputs), vp,
                                       C.POINTER(sz), C.POINTER(Record)]
        L.zk_vm_trace.argtypes = [C.c_char_p, vp, sz, vp, sz, u32, u32, vp, vp, sz, C.POINTER(sz), vp, vp]
        L.zk_vm_last_error.restype = C.c_char_p
        L.zk_program_compile.argtypes = [C.c_char_p, C.POINTER(vp), vp, C.POINTER(sz)]
        L.zk_program_trace.argtypes = [vp, vp, sz, vp, sz, u32, u32, vp, vp, sz, C.POINTER(sz), vp]
        L.zk_vm_trace_device.argtypes = [vp, vp, vp, sz, vp, sz, u32, u32, vp, C.POINTER(sz), vp]
        L.zk_vm_prove.argtypes = [vp, vp, vp, sz, vp, sz, u32, u32, vp, C.POINTER(Options), vp, C.POINTER(sz), vp, vp]
        L.zk_vm_prove_sharded.argtypes = [vp, vp, C.c_int, vp, vp, sz, vp, sz, u32, u32, vp, C.POINTER(Options), vp,
                                          C.POINTER(sz), vp, vp]
        L.zk_diag_vm_states.argtypes = [vp, vp, sz, vp, sz, u32, u32, sz, sz, vp, vp]
        L.zk_program_free.argtypes = [vp]
        L.zk_program_free.restype = None
        L.zk_diag_mul_limbs_host.argtypes = [vp, vp, vp, sz]
        L.zk_diag_mul_limbs_host.restype = None
        L.zk_diag_dot_host.argtypes = [vp, vp, sz, vp]
        L.zk_diag_dot_host.restype = None
        L.zk_diag_blake3_host.argtypes = [vp, sz, vp]
        L.zk_diag_blake3_host.restype = None
        L.zk_diag_field_op.argtypes = [i32, i32, vp, vp, vp, sz]
        L.zk_diag_blake3_rows.argtypes = [i32, vp, i32, sz, vp]
        L.zk_diag_ntt.argtypes = [i32, vp, sz, i32, i32, vp, vp]
        _lib = L
    return _lib


def check(rc: int, what: str = ""):
    if rc != ZK_OK:
        msg = lib().zk_last_error()
        raise ZkError(rc, f"{what}: {msg.decode() if msg else ''}")


def device_count() -> int:
    c = C.c_int(0)
    lib().zk_device_count(C.byref(c))
    return c.value


def pci_bus_id(device: int) -> str:
    buf = C.create_string_buffer(32)
    check(lib().zk_device_pci_bus_id(device, buf, len(buf)), "zk_device_pci_bus_id")
    return buf.value.decode()


def synchronize(device: int):
    check(lib().zk_device_synchronize(device), "zk_device_synchronize")


def hip_runtime():
    """ctypes handle of the HIP runtime the library runs on (the same mapped file: dlopen returns its handle)."""
    path = runtime_info()["hip_runtime"]
    h = C.CDLL(path)
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    return h
