"""zkvm_amd -- MI355X (gfx950) STARK prover for the Encrypt-zkVM execution trace.

Product path: libzkvm_gpu.so (HIP kernels + C ABI, include/zkvm_gpu.h) driven through
`zkvm_amd.prover`.  `zkvm_amd.workloads` builds seeded synthetic programs and inputs.
"""
from .native import ZkError, device_count  # noqa: F401
from .prover import (REFERENCE_OPTIONS, ExecutionProver, GpuProver, ProofOptions,  # noqa: F401
                     make_pub_inputs, prove, vm_trace)
