// runtime.cpp -- what the host needs from the HIP runtime and RCCL the library itself is linked against, so that a
// host process never has to load a second copy of either (bench.py and the tests are torch-free: torch bundles its own
// libamdhip64 / librccl, and glibc would satisfy this library's DT_NEEDED entries with whichever copy came first).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>

#include "../../include/zkvm_gpu.h"
#include "prover_internal.hpp"

int zk_runtime_versions(int *hip_runtime, int *rccl) {
    int h = 0, r = 0;
    ZK_CHECK_HIP(hipRuntimeGetVersion(&h));
    const ncclResult_t nr = ncclGetVersion(&r);
    if (nr != ncclSuccess) ZK_FAIL(ZK_ERR_DEVICE, std::string("ncclGetVersion: ") + ncclGetErrorString(nr));
    if (hip_runtime) *hip_runtime = h;
    if (rccl) *rccl = r;
    return ZK_OK;
}

int zk_device_pci_bus_id(int device, char *bus_id, int len) {
    if (!bus_id || len < 13) ZK_FAIL(ZK_ERR_INVALID_ARG, "bus_id needs room for 13 bytes (dddd:bb:dd.f)");
    ZK_CHECK_HIP(hipDeviceGetPCIBusId(bus_id, len, device));
    return ZK_OK;
}

int zk_device_synchronize(int device) {
    ZK_CHECK_HIP(hipSetDevice(device));
    ZK_CHECK_HIP(hipDeviceSynchronize());
    return ZK_OK;
}
