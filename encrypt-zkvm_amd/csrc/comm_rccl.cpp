// comm_rccl.cpp -- zk_comm over RCCL (xGMI within a node): one process per GPU.  The collectives run on the stream
// shard.hip hands in (the prover's exchange stream, ordered after its compute stream by an event), so they overlap
// the compute that does not wait for them.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>

#include "../../include/zkvm_gpu.h"
#include "comm.hpp"
#include "prover_internal.hpp"

namespace {

struct RcclComm : zk_comm {
    ncclComm_t comm = nullptr;
    ~RcclComm() override {
        if (comm) ncclCommDestroy(comm);
    }
    bool loopback() const override { return false; }
    int all_to_all(const std::vector<zk_prover *> &P, const std::vector<const void *> &send,
                   const std::vector<void *> &recv, size_t bytes, hipStream_t is) override {
        if (P.size() != 1) ZK_FAIL(ZK_ERR_INVALID_ARG, "an RCCL communicator drives exactly one local rank");
        ncclResult_t r = ncclAllToAll(send[0], recv[0], bytes, ncclUint8, comm, is);
        if (r != ncclSuccess) ZK_FAIL(ZK_ERR_DEVICE, std::string("ncclAllToAll: ") + ncclGetErrorString(r));
        return ZK_OK;
    }
    int all_gather(const std::vector<zk_prover *> &P, const std::vector<const void *> &send,
                   const std::vector<void *> &recv, size_t bytes, hipStream_t is) override {
        if (P.size() != 1) ZK_FAIL(ZK_ERR_INVALID_ARG, "an RCCL communicator drives exactly one local rank");
        ncclResult_t r = ncclAllGather(send[0], recv[0], bytes, ncclUint8, comm, is);
        if (r != ncclSuccess) ZK_FAIL(ZK_ERR_DEVICE, std::string("ncclAllGather: ") + ncclGetErrorString(r));
        return ZK_OK;
    }
};

}  // namespace

int zk_rccl_unique_id(unsigned char id[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) ZK_FAIL(ZK_ERR_DEVICE, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    memcpy(id, &u, 128);
    return ZK_OK;
}

int zk_make_rccl_comm(const unsigned char id[128], int rank, int world, int device, zk_comm **out) {
    ZK_CHECK_HIP(hipSetDevice(device));
    ncclUniqueId u;
    memcpy(&u, id, 128);
    auto *c = new RcclComm();
    c->world = world;
    c->rank = rank;
    ncclResult_t r = ncclCommInitRank(&c->comm, world, u, rank);
    if (r != ncclSuccess) {
        delete c;
        ZK_FAIL(ZK_ERR_DEVICE, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    *out = c;
    return ZK_OK;
}
