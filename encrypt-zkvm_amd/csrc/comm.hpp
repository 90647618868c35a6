// comm.hpp -- the exchange steps of the coset-sharded prover (shard.hip).
//
// A zk_comm connects `world` ranks; each rank proves with one zk_prover (one GPU).  A process drives either every
// rank (loopback: in-process copies, for tests and single-node emulation) or exactly one (RCCL over xGMI, one process
// per GPU; or a caller transport).  A collective is issued on ONE stream, `is`, that the caller (shard.hip
// xchg_start) has already ordered after every local rank's compute stream; the caller records the completion on it
// and makes the consumers wait (xchg_wait), so the exchange overlaps whatever compute does not need it.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include <vector>

struct zk_prover;

struct zk_comm {
    int world = 1;
    int rank = 0;  // the rank this process drives (RCCL); loopback drives 0 .. world-1
    bool measure = false;  // loopback only: the serialised measurement mode (zk_comm_set_measure)
    int split_rep = -1;    // zk_comm_set_trace_split: trace columns every rank interpolates itself (-1: by world)
    virtual ~zk_comm() {}
    virtual bool loopback() const = 0;
    // for every local rank l: send[l] holds `world` chunks of `bytes` (chunk d goes to rank d);
    // recv[l] receives `world` chunks (chunk s came from rank s)
    virtual int all_to_all(const std::vector<zk_prover *> &P, const std::vector<const void *> &send,
                           const std::vector<void *> &recv, size_t bytes, hipStream_t is) = 0;
    // recv[l] = chunk of rank 0 || chunk of rank 1 || ... (each `bytes`); send[l] = this rank's chunk
    virtual int all_gather(const std::vector<zk_prover *> &P, const std::vector<const void *> &send,
                           const std::vector<void *> &recv, size_t bytes, hipStream_t is) = 0;
};

// defined in comm_rccl.cpp (links librccl)
int zk_make_rccl_comm(const unsigned char id[128], int rank, int world, int device, zk_comm **out);
int zk_rccl_unique_id(unsigned char id[128]);
