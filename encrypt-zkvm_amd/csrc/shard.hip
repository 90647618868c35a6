// shard.hip -- one proof with the LDE domain sharded by coset over `world` GPUs.
//
// Rank g of G owns the LDE cosets r = g*Bl + j, j < Bl = 8/G (blowup 8; round 6: a block, so that the Merkle leaves
// 8q + r of a group q that one rank holds are siblings).  Per stage:
//   trace interpolation          host trace: split by column (a rank uploads and interpolates W/G columns,
//                                round robin), in-place all-gathers of the coefficients; device trace: replicated
//   trace LDE, constraint eval,  local: a coset's LDE is an independent size-n NTT, and constraint
//   DEEP LDE, first FRI fold     row i+8 / a fold row {e[r' + k N/fold]} stay inside one coset
//   OOD values, DEEP coefficients  split by coefficient range; all-gathers of partial sums / range totals and of
//                                the quotient slices
//   Merkle trees                 each rank hashes its leaves and their subtree up to its block of Bl siblings,
//   (trace, composition, FRI 0)  all-to-all of the block nodes into contiguous ranges, a local subtree per rank,
//                                all-gather of the G subtree roots
//   composition interpolation    per-coset inverse NTT local; all-to-all of coefficient slices for the
//                                cross-coset radix-8 step; all-gather of the 7 column polynomials
//   FRI layers 1, >= 2           layer 1 as layer 0 (block trees, local fold), all-gather of layer 2, then the
//                                rest on the lead rank (small)
//   openings                     every rank gathers what it owns, all-gather, the host combines
// The Fiat-Shamir transcript runs on every process's host over identical (all-gathered) roots, so no
// challenge is ever broadcast.  The proof bytes equal the single-GPU prover's (tests/test_sharded.py).
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "blake3.hpp"
#include "comm.hpp"
#include "fri_small.hpp"
#include "host_pool.hpp"
#include "prover_internal.hpp"

using namespace zk;

namespace {

static inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

// ---------------------------------------------------------------- loopback communicator
// Every rank in this process: the collective is device-to-device copies, all of them on the issue stream (ordered
// after every rank's compute stream by xchg_start), so its completion covers every rank's reads and writes.
struct LoopbackComm : zk_comm {
    bool loopback() const override { return true; }
    int all_to_all(const std::vector<zk_prover *> &P, const std::vector<const void *> &send,
                   const std::vector<void *> &recv, size_t bytes, hipStream_t is) override {
        if ((int)P.size() != world) ZK_FAIL(ZK_ERR_INVALID_ARG, "a loopback communicator drives every rank");
        for (int d = 0; d < world; d++)
            for (int s = 0; s < world; s++)
                ZK_CHECK_HIP(hipMemcpyAsync((uint8_t *)recv[d] + s * bytes, (const uint8_t *)send[s] + d * bytes, bytes,
                                            hipMemcpyDeviceToDevice, is));
        return ZK_OK;
    }
    int all_gather(const std::vector<zk_prover *> &P, const std::vector<const void *> &send,
                   const std::vector<void *> &recv, size_t bytes, hipStream_t is) override {
        if ((int)P.size() != world) ZK_FAIL(ZK_ERR_INVALID_ARG, "a loopback communicator drives every rank");
        for (int d = 0; d < world; d++)
            for (int s = 0; s < world; s++)
                if ((uint8_t *)recv[d] + s * bytes != send[s])  // in place: a rank's own chunk is already there
                    ZK_CHECK_HIP(hipMemcpyAsync((uint8_t *)recv[d] + s * bytes, send[s], bytes, hipMemcpyDeviceToDevice, is));
        return ZK_OK;
    }
};

// ---------------------------------------------------------------- caller-transport communicator
// One rank per process, exchanges through a caller callback over host memory (MPI, gloo, TCP across nodes).  The
// staging is synchronous on the host: device chunk -> host on the issue stream, callback, host -> device.
struct HostComm : zk_comm {
    zk_exchange_fn fn = nullptr;
    void *ctx = nullptr;
    std::vector<uint8_t> sbuf, rbuf;
    bool loopback() const override { return false; }
    int run(const std::vector<zk_prover *> &P, int op, const void *send, size_t sbytes, void *recv, size_t bytes,
            hipStream_t is) {
        if (P.size() != 1) ZK_FAIL(ZK_ERR_INVALID_ARG, "a host-exchange communicator drives exactly one local rank");
        const size_t rbytes = bytes * (size_t)world;
        sbuf.resize(std::max<size_t>(sbytes, 1));
        rbuf.resize(std::max<size_t>(rbytes, 1));
        if (sbytes) ZK_CHECK_HIP(hipMemcpyAsync(sbuf.data(), send, sbytes, hipMemcpyDeviceToHost, is));
        ZK_CHECK_HIP(hipStreamSynchronize(is));
        const int rc = fn(ctx, op, sbuf.data(), rbuf.data(), bytes);
        if (rc != 0) ZK_FAIL(ZK_ERR_DEVICE, "exchange callback failed (" + std::to_string(rc) + ")");
        if (rbytes) ZK_CHECK_HIP(hipMemcpyAsync(recv, rbuf.data(), rbytes, hipMemcpyHostToDevice, is));
        ZK_CHECK_HIP(hipStreamSynchronize(is));  // rbuf is reused by the next exchange
        return ZK_OK;
    }
    int all_to_all(const std::vector<zk_prover *> &P, const std::vector<const void *> &send,
                   const std::vector<void *> &recv, size_t bytes, hipStream_t is) override {
        return run(P, ZK_XCHG_ALL_TO_ALL, send.at(0), bytes * (size_t)world, recv.at(0), bytes, is);
    }
    int all_gather(const std::vector<zk_prover *> &P, const std::vector<const void *> &send,
                   const std::vector<void *> &recv, size_t bytes, hipStream_t is) override {
        return run(P, ZK_XCHG_ALL_GATHER, send.at(0), bytes, recv.at(0), bytes, is);
    }
};

// ---------------------------------------------------------------- local-coset kernels
__device__ __forceinline__ void st_digest(uint8_t *dst, const uint32_t h[8]) {
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    d[0] = make_uint4(h[0], h[1], h[2], h[3]);
    d[1] = make_uint4(h[4], h[5], h[6], h[7]);
}
// Block ownership (round 6): rank g owns the cosets g Bl .. g Bl + Bl - 1, so in every group q of 8 consecutive leaves
// 8q .. 8q + 7 (leaf 8q + r: row q of coset r) its Bl leaves are siblings: it hashes them and their subtree up to level
// Lb = log2 Bl itself, and only that block node -- 1/Bl of the leaf digests -- crosses the link.  Each tree keeps the
// levels 0 .. Lb of its own leaves in a block buffer (level l: node (q, i) at lvl_off(l) + q (Bl >> l) + i, for the
// openings) and sends the block nodes out in K pieces: piece k holds, for every destination d, the groups
// q = d QG + k QGK + q'' (QG = Q / G groups per destination, QGK = QG / K), in send order [d][q''].
__device__ __forceinline__ size_t blk_group(size_t t, int log_QG, int log_K, int k) {
    const int log_QGK = log_QG - log_K;
    const size_t qq = t & (((size_t)1 << log_QGK) - 1), d = t >> log_QGK;
    return (d << log_QG) + ((size_t)k << log_QGK) + qq;
}
// the Bl leaves of group q (leaf(j, h): local coset slot j), their subtree into blk, the block node into send_slot
template <int BL, typename Leaf>
__device__ __forceinline__ void blk_levels(size_t Q, size_t q, uint8_t *blk, uint8_t *send_slot, Leaf leaf) {
    static_assert(BL == 1 || BL == 2 || BL == 4, "a sharded rank holds 1, 2 or 4 cosets");
    uint32_t a[8];
    leaf(0, a);
    st_digest(blk + 32 * (q * BL), a);
    if constexpr (BL >= 2) {
        uint32_t b[8];
        leaf(1, b);
        st_digest(blk + 32 * (q * BL + 1), b);
        b3::merge(a, b, a);
        st_digest(blk + 32 * (Q * BL + q * (BL / 2)), a);
        if constexpr (BL == 4) {
            uint32_t c[8], d[8];
            leaf(2, c);
            st_digest(blk + 32 * (q * 4 + 2), c);
            leaf(3, d);
            st_digest(blk + 32 * (q * 4 + 3), d);
            b3::merge(c, d, c);
            st_digest(blk + 32 * (Q * 4 + q * 2 + 1), c);
            b3::merge(a, c, a);
            st_digest(blk + 32 * (Q * 6 + q), a);
        }
    }
    st_digest(send_slot, a);
}

// LDE rows (column c, local coset j at base[(c*Bl + j)*n + q]; Q = n groups): piece k of K
template <int BL>
__global__ void __launch_bounds__(256) k_sh_hash_rows_blk(const fe *base, int ncols, int log_n, int log_QG, int log_K,
                                                          int k, uint8_t *blk, uint8_t *send) {
    const size_t n = (size_t)1 << log_n;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= (n >> log_K)) return;
    const size_t q = blk_group(t, log_QG, log_K, k), cs = (size_t)BL * n;
    blk_levels<BL>(n, q, blk, send + 32 * t, [&](int j, uint32_t h[8]) {
        const fe *p = base + (size_t)j * n + q;
        b3::hash_elements(ncols, [&](int c) { return p[(size_t)c * cs]; }, h);
    });
}

// FRI layer-0 leaves (Q = m groups): leaf (j, q0) holds deep[j][q0 + k m], k < fold (KX planes at stride Bl n)
template <int BL, int KX>
__global__ void __launch_bounds__(256) k_sh_hash_fri0_blk(const fe *deep, int log_n, int fold, int log_m, int log_QG,
                                                          int log_K, int kp, uint8_t *blk, uint8_t *send) {
    const size_t n = (size_t)1 << log_n, m = (size_t)1 << log_m, cs = (size_t)BL * n;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= (m >> log_K)) return;
    const size_t q = blk_group(t, log_QG, log_K, kp);
    blk_levels<BL>(m, q, blk, send + 32 * t, [&](int j, uint32_t h[8]) {
        const fe *p = deep + (size_t)j * n + q;
        if constexpr (KX == 1)
            b3::hash_elements(fold, [&](int e) { return p[(size_t)e << log_m]; }, h);
        else
            b3::hash_elements(2 * fold, [&](int e) { return p[(size_t)(e & 1) * cs + ((size_t)(e >> 1) << log_m)]; }, h);
    });
}

template <int BL>
static void launch_fri0_blk(hipStream_t st, int KX, const fe *deep, int log_n, int fold, int log_m, int log_QG,
                            int log_K, int k, uint8_t *blk, uint8_t *send) {
    const dim3 grid(cdiv(((size_t)1 << log_m) >> log_K, 256));
    if (KX == 1)
        hipLaunchKernelGGL((k_sh_hash_fri0_blk<BL, 1>), grid, dim3(256), 0, st, deep, log_n, fold, log_m, log_QG, log_K, k,
                           blk, send);
    else
        hipLaunchKernelGGL((k_sh_hash_fri0_blk<BL, 2>), grid, dim3(256), 0, st, deep, log_n, fold, log_m, log_QG, log_K, k,
                           blk, send);
}

// piece k's received block nodes [s][q''] (group q' = k QGK + q'' of source s is level-Lb node q' G + s of this rank's
// subtree) merged straight into their parents: level Lb + 1 node q' G/2 + j = merge(node q' G + 2j, node q' G + 2j + 1),
// into lvl1 (j fastest: the stores are contiguous, the loads 32-B runs of G/2 chunks)
__global__ void k_sh_blk_merge(const uint8_t *recv, int G, int log_QGK, int k, uint8_t *lvl1) {
    const int hg = G / 2, log_hg = G >= 4 ? (G >= 8 ? 2 : 1) : 0;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= ((size_t)hg << log_QGK)) return;
    const size_t j = t & (size_t)(hg - 1), qq = t >> log_hg;
    uint32_t l[8], r[8], h[8];
    const uint4 *a = reinterpret_cast<const uint4 *>(recv + 32 * (((2 * j) << log_QGK) + qq));
    const uint4 *c = reinterpret_cast<const uint4 *>(recv + 32 * (((2 * j + 1) << log_QGK) + qq));
    const uint4 a0 = a[0], a1 = a[1], c0 = c[0], c1 = c[1];
    l[0] = a0.x; l[1] = a0.y; l[2] = a0.z; l[3] = a0.w; l[4] = a1.x; l[5] = a1.y; l[6] = a1.z; l[7] = a1.w;
    r[0] = c0.x; r[1] = c0.y; r[2] = c0.z; r[3] = c0.w; r[4] = c1.x; r[5] = c1.y; r[6] = c1.z; r[7] = c1.w;
    b3::merge(l, r, h);
    st_digest(lvl1 + 32 * ((((size_t)k << log_QGK) + qq) * hg + j), h);
}

// all-gathered chunks [s][j][q'] (source chunk s at item s * src_stride) -> natural order: item (s Bl + j) + 8 q' (local
// coset j of rank s is coset s Bl + j).  src_stride > Bl << log_mg when each source sent several planes.
__global__ void k_sh_permute(const uint8_t *recv, int G, int Bl, int log_mg, int esize, size_t src_stride,
                             uint8_t *out) {
    const size_t per = (size_t)Bl << log_mg;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= per * G) return;
    const size_t s = t / per, rem = t % per, j = rem >> log_mg, qp = rem & (((size_t)1 << log_mg) - 1);
    const size_t idx = (s * Bl + j) + 8 * qp;
    const uint4 *src = reinterpret_cast<const uint4 *>(recv + (s * src_stride + rem) * esize);
    uint4 *dst = reinterpret_cast<uint4 *>(out + idx * esize);
    for (int w = 0; w < esize / 16; w++) dst[w] = src[w];
}

// one coset's coefficient slices (KX planes at plane_stride) for its all-to-all: send[d][plane][k'] = c[plane][d*kg + k']
__global__ void k_sh_pack_coset(const fe *c, size_t plane_stride, int log_n, int KX, int log_kg, fe *send) {
    const size_t n = (size_t)1 << log_n;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= (size_t)KX * n) return;
    const size_t pln = t >> log_n, k = t & (n - 1);
    send[((((k >> log_kg) * KX) + pln) << log_kg) + (k & (((size_t)1 << log_kg) - 1))] = c[pln * plane_stride + k];
}

// first FRI fold over the local cosets: row r' = r + 8*q0 (values deep[j][q0 + k*m]) -> out[j*m + q0], as the
// single-GPU fold (kernels.hip k_fri_fold: idft_small, then Horner at beta = alpha / x_r')
template <int F>
__global__ void __launch_bounds__(256) k_sh_fri_fold0(const fe *deep, int log_n, int Bl, int g, int log_m,
                                                      const FoldConsts *Fc, const fe *wi_lo, const fe *wi_hi,
                                                      size_t wstride, fe *out) {
    const size_t n = (size_t)1 << log_n, m = (size_t)1 << log_m;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= ((size_t)Bl << log_m)) return;
    const size_t j = t >> log_m, q0 = t & (m - 1);
    const size_t rp = (size_t)(g * Bl + (int)j) + 8 * q0;  // row index in the layer (1/x_r: w_N^-(rp wstride))
    const size_t wi = rp * wstride;
    fe v[F];
#pragma unroll
    for (int k = 0; k < F; k++) v[k] = deep[j * n + q0 + ((size_t)k << log_m)];
    const fe beta = fe_mul(Fc->alpha, fe_mul(Fc->inv_offset, fe_mul(wi_lo[wi & 2047], wi_hi[wi >> 11])));
    idft_small<F>(v, Fc->zinv);
    fe acc = v[F - 1];
#pragma unroll
    for (int mm = F - 2; mm >= 0; mm--) acc = fe_add(fe_mul(acc, beta), v[mm]);
    out[t] = fe_mul(acc, Fc->inv_fold);
}

// ---- FieldExtension::Quadratic versions: E buffers are planar with plane stride Bl*n (DEEP) / Bl*m (fold)
template <int F>
__global__ void __launch_bounds__(256) k_sh_fri_fold0_ext(const fe *deep, int log_n, int Bl, int g, int log_m,
                                                          const FoldConstsE *Fc, const fe *wi_lo, const fe *wi_hi,
                                                          size_t wstride, fe *out) {
    const size_t n = (size_t)1 << log_n, m = (size_t)1 << log_m, cs = (size_t)Bl * n, om = (size_t)Bl * m;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= om) return;
    const size_t j = t >> log_m, q0 = t & (m - 1);
    const size_t rp = (size_t)(g * Bl + (int)j) + 8 * q0, wi = rp * wstride;
    fe va[F], vb[F];
#pragma unroll
    for (int k = 0; k < F; k++) {
        va[k] = deep[j * n + q0 + ((size_t)k << log_m)];
        vb[k] = deep[cs + j * n + q0 + ((size_t)k << log_m)];
    }
    const fe2 beta = fe2_mulb(Fc->alpha, fe_mul(Fc->inv_offset, fe_mul(wi_lo[wi & 2047], wi_hi[wi >> 11])));
    idft_small<F>(va, Fc->zinv);
    idft_small<F>(vb, Fc->zinv);
    fe2 acc = fe2{va[F - 1], vb[F - 1]};
#pragma unroll
    for (int mm = F - 2; mm >= 0; mm--) acc = fe2_add(fe2_mul(acc, beta), fe2{va[mm], vb[mm]});
    acc = fe2_mulb(acc, Fc->inv_fold);
    out[t] = acc.a;
    out[om + t] = acc.b;
}

// a fold over the local cosets (layer 0, or layer 1 with wstride = fold) for fold 2 / 4 / 8 / 16 (KX planes)
static void sh_fri_fold0(hipStream_t st, int KX, int fold, const fe *deep, int log_n, int Bl, int g, int log_m,
                         const void *consts, const fe *wi_lo, const fe *wi_hi, size_t wstride, fe *out) {
    const dim3 grid(cdiv((size_t)Bl << log_m, 256));
#define ZK_SH_FOLD(FF)                                                                                              \
    do {                                                                                                            \
        if (KX == 1)                                                                                                \
            hipLaunchKernelGGL(k_sh_fri_fold0<FF>, grid, dim3(256), 0, st, deep, log_n, Bl, g, log_m,               \
                               (const FoldConsts *)consts, wi_lo, wi_hi, wstride, out);                             \
        else                                                                                                        \
            hipLaunchKernelGGL(k_sh_fri_fold0_ext<FF>, grid, dim3(256), 0, st, deep, log_n, Bl, g, log_m,           \
                               (const FoldConstsE *)consts, wi_lo, wi_hi, wstride, out);                            \
    } while (0)
    switch (fold) {
        case 2: ZK_SH_FOLD(2); break;
        case 4: ZK_SH_FOLD(4); break;
        case 8: ZK_SH_FOLD(8); break;
        default: ZK_SH_FOLD(16); break;
    }
#undef ZK_SH_FOLD
}

// the suffix carried into rank `rank`'s DEEP range: out[c] = sum over later ranks h of all[h * nc + c]
__global__ void k_sh_suffix_carry(const fe *all, int G, int rank, int nc, fe *out) {
    const int c = threadIdx.x;
    if (c >= nc) return;
    fe s = fe_zero();
    for (int h = rank + 1; h < G; h++) s = fe_add(s, all[(size_t)h * nc + c]);
    out[c] = s;
}

// ---------------------------------------------------------------- a Merkle tree split over G ranks
// M leaves in natural order (leaf 8q + r: group q, coset r).  Levels 0 .. Lb (Lb = log2 Bl) live in each coset owner's
// block buffer (blk_levels); above them rank d holds the subtree over level-Lb nodes [d Q, (d+1) Q) (Q = M / 8), as a
// heap `nodes` (level Lb + 1 at [Q/2, Q), ..., its root at 1); the top (G subtree roots) is kept on the host.
struct DistTree {
    size_t M = 0, Mr = 0, Q = 0;
    int G = 1, Bl = 1, Lb = 0;
    std::vector<uint8_t *> blk, nodes;               // per local rank
    std::vector<std::array<uint8_t, 32>> top;        // heap nodes 1 .. 2G-1
    uint8_t root[32];
    // chunk source of global leaf idx (is_node 0) or heap node idx (leaves are M + i): owner rank, buffer (1 subtree
    // nodes, 2 block buffer), byte offset; owner -1 = host top node (copied into `host`)
    struct Loc {
        int owner;
        int which;
        size_t off;
    };
    size_t lvl_off(int l) const {  // level l's first node in a block buffer
        size_t o = 0;
        for (int t = 0; t < l; t++) o += Q * (size_t)(Bl >> t);
        return o;
    }
    Loc locate(int is_node, uint64_t idx) const {
        int L = 0;
        uint64_t i = idx;
        if (is_node) {
            L = 1;
            while ((M >> L) > idx) L++;
            i = idx - (M >> L);
        }
        if (L <= Lb) {  // a block level: on the owner of the node's cosets
            const uint64_t per = (uint64_t)8 >> L, bl = (uint64_t)Bl >> L, q = i / per, rr = i % per;
            return {(int)(rr / bl), 2, 32 * (lvl_off(L) + q * bl + rr % bl)};
        }
        const size_t c = Mr >> L;
        if (c == 0) return {-1, 0, 32 * idx};
        return {(int)(i / c), 1, 32 * (c + i % c)};
    }
};

struct Ctx {
    zk_comm *comm;
    std::vector<zk_prover *> P;
    std::vector<int> rank;  // rank of each local prover
    std::vector<Plan *> pl;
    int G, Bl, log_n, C;
    size_t n;
    // zk_vm_prove_sharded: the preprocessed columns of each local rank (its own cosets), or null: the device trace
    // then holds only the dynamic stack columns 12 .. 12 + md - 1
    const FixedCols *fixed = nullptr;
    // host traces: the previous proof's column hints may be used (hint_ok); whether this proof derives the clock
    // (sh_clock), and the hinted columns the ranks' checks refuted (sh_refuted, bit c: prove_sharded returned
    // ZK_SH_REDO, and prove_sharded_entry proves again without hints)
    bool hint_ok = true, sh_clock = false;
    uint32_t sh_refuted = 0;
    bool lead_seg = false;  // the schedule segment being enqueued runs on the lead rank only (lead_segment)
};
constexpr int ZK_SH_REDO = 1000;  // (internal) a refuted column hint voided the proof on every rank


// ---------------------------------------------------------------- exchanges, overlapped with compute (round 6)
// xchg_start issues a collective on the exchange stream of local rank 0 (its own stream per process: RCCL, host
// transport; every rank's copies for the loopback), ordered after everything already enqueued on every local rank's
// compute stream (an event per rank), and records its completion; xchg_wait makes every local compute stream wait
// for that completion -- a device-side wait, enqueued after the completion was recorded, so it never parks a
// queue on an event not yet recorded.  Between the two the compute streams run whatever does not read the received
// data or write the sent data (the callers keep to that).  xchg = start + wait.  Timing: events around the collective
// on its stream (total) and around the wait on rank 0's compute stream (exposed), and the schedule log
// (zk_prover_shard_schedule) of every start, wait and segment boundary.
// Measurement mode (zk_comm_set_measure, loopback): every rank's compute and the copies share rank 0's stream.
enum XOp { A2A, AG };
struct XH {
    int idx = -1;
};
static int pool_events(zk_prover *p, size_t k, size_t *first) {
    while (p->xchg_pool.size() < p->xchg_next + k) {
        hipEvent_t ev;
        ZK_CHECK_HIP(hipEventCreate(&ev));
        p->xchg_pool.push_back(ev);
    }
    *first = p->xchg_next;
    p->xchg_next += k;
    return ZK_OK;
}
static int exchange_stream(zk_prover *p, hipStream_t *out) {
    if (!p->cst) {
        // the highest priority the device offers: an RCCL collective's workgroups are dispatched ahead of the queued
        // workgroups of the compute stream's long launches instead of behind them
        int least = 0, greatest = 0;
        ZK_CHECK_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        ZK_CHECK_HIP(hipStreamCreateWithPriority(&p->cst, hipStreamNonBlocking, greatest));
    }
    if (!p->ev_ready) ZK_CHECK_HIP(hipEventCreateWithFlags(&p->ev_ready, hipEventDisableTiming));
    *out = p->cst;
    return ZK_OK;
}
// a schedule entry on local rank 0's compute stream: kind 'S' / 'W' (exchange x) or 'K' (segment boundary);
// `lead`: the segment ending here ran on the lead rank only
static int sched_entry(Ctx &X, char kind, int x, bool post_now = true) {
    zk_prover *p = X.P[0];
    size_t e;
    ZK_TRY(pool_events(p, 2, &e));
    ZK_CHECK_HIP(hipEventRecord(p->xchg_pool[e], p->st));
    if (post_now) ZK_CHECK_HIP(hipEventRecord(p->xchg_pool[e + 1], p->st));
    p->sched.push_back({kind, x, e, e + 1, X.lead_seg});
    X.lead_seg = false;
    return ZK_OK;
}
// the segment starting here runs on the lead rank only (until the next entry)
static int lead_segment(Ctx &X) {
    ZK_TRY(sched_entry(X, 'K', -1));
    X.lead_seg = true;
    return ZK_OK;
}
int xchg_start(Ctx &X, const char *name, XOp op, const std::vector<const void *> &snd, const std::vector<void *> &rcv,
               size_t bytes, XH *h) {
    zk_prover *p0 = X.P[0];
    ZK_CHECK_HIP(hipSetDevice(p0->device));
    size_t e;
    ZK_TRY(pool_events(p0, 4, &e));
    const int x = (int)p0->xchg.size();
    p0->xchg.push_back({name, (double)bytes * (X.G - 1), e, op == A2A ? 0 : 1, false});
    hipStream_t is;
    if (X.comm->measure) {
        is = p0->st;  // every rank's stream is this one (prove_sharded_entry): program order, no overlap
        ZK_TRY(sched_entry(X, 'S', x, false));
    } else {
        ZK_TRY(exchange_stream(p0, &is));
        ZK_TRY(sched_entry(X, 'S', x));
        for (zk_prover *p : X.P) {
            ZK_CHECK_HIP(hipSetDevice(p->device));
            if (!p->ev_ready) ZK_CHECK_HIP(hipEventCreateWithFlags(&p->ev_ready, hipEventDisableTiming));
            ZK_CHECK_HIP(hipEventRecord(p->ev_ready, p->st));
            ZK_CHECK_HIP(hipStreamWaitEvent(is, p->ev_ready, 0));  // (captured now: the event may be recorded again)
        }
        ZK_CHECK_HIP(hipSetDevice(p0->device));
    }
    ZK_CHECK_HIP(hipEventRecord(p0->xchg_pool[e], is));
    ZK_TRY(op == A2A ? X.comm->all_to_all(X.P, snd, rcv, bytes, is) : X.comm->all_gather(X.P, snd, rcv, bytes, is));
    ZK_CHECK_HIP(hipSetDevice(p0->device));
    ZK_CHECK_HIP(hipEventRecord(p0->xchg_pool[e + 1], is));
    if (X.comm->measure) ZK_CHECK_HIP(hipEventRecord(p0->xchg_pool[p0->sched.back().post], p0->st));
    h->idx = x;
    return ZK_OK;
}
int xchg_wait(Ctx &X, XH &h) {
    if (h.idx < 0) return ZK_OK;
    zk_prover *p0 = X.P[0];
    auto &r = p0->xchg[h.idx];
    const int x = h.idx;
    h.idx = -1;
    if (r.waited) return ZK_OK;
    r.waited = true;
    ZK_CHECK_HIP(hipSetDevice(p0->device));
    ZK_CHECK_HIP(hipEventRecord(p0->xchg_pool[r.ev + 2], p0->st));
    ZK_TRY(sched_entry(X, 'W', x, false));
    if (!X.comm->measure)
        for (zk_prover *p : X.P) {
            ZK_CHECK_HIP(hipSetDevice(p->device));
            ZK_CHECK_HIP(hipStreamWaitEvent(p->st, p0->xchg_pool[r.ev + 1], 0));
        }
    ZK_CHECK_HIP(hipSetDevice(p0->device));
    ZK_CHECK_HIP(hipEventRecord(p0->xchg_pool[r.ev + 3], p0->st));
    ZK_CHECK_HIP(hipEventRecord(p0->xchg_pool[p0->sched.back().post], p0->st));
    return ZK_OK;
}
int xchg(Ctx &X, const char *name, XOp op, const std::vector<const void *> &snd, const std::vector<void *> &rcv,
         size_t bytes) {
    XH h;
    ZK_TRY(xchg_start(X, name, op, snd, rcv, bytes, &h));
    return xchg_wait(X, h);
}

// the block levels (the hash kernel: leaves, their subtree up to Lb into blk, block nodes into the send scratch in piece
// order), all-to-all of the block nodes, merged on arrival into level Lb + 1 of the subtree, the subtree, roots.  The
// block nodes go out in K pieces: piece k's all-to-all runs on the exchange stream while piece k + 1 is hashed.
// hash(l, send, log_QG, log_K, k) launches piece k of local rank l.  `rows`: the leaves are LDE rows (7 or 2 BLAKE3
// blocks each), whose hashing the pieces hide; the FRI trees' leaves hash in a fraction of that and go in one piece.
template <typename HashFn>
int dist_commit(Ctx &X, DistTree &T, size_t M, HashFn hash, const std::vector<uint8_t *> &scratch,
                const std::vector<uint8_t *> &blk, const std::vector<uint8_t *> &nodes, const char *digests_name,
                const char *roots_name, bool rows = true) {
    const int nl = (int)X.P.size();
    T.M = M;
    T.G = X.G;
    T.Mr = M / X.G;
    T.Q = M / 8;
    T.Bl = X.Bl;
    T.Lb = ilog2((size_t)X.Bl);
    T.blk = blk;
    T.nodes = nodes;
    const size_t Q = T.Q, QG = Q / X.G;  // groups per destination rank
    const int log_QG = ilog2(QG);
    // pieces only where the transfer outweighs the latency of three more collectives: >= 1 MiB per destination and
    // piece (the trace and composition trees at 2^20 and up; small FRI trees go in one piece)
    const int log_K = rows && QG >= ((size_t)1 << 17) ? 2 : 0, K = 1 << log_K;
    const int log_QGK = log_QG - log_K;
    const size_t piece = 32 * (size_t)X.G << log_QGK;  // bytes of one piece (all destinations)
    std::vector<XH> h(K);
    std::vector<const void *> snd(nl);
    std::vector<void *> rcv(nl);
    for (int k = 0; k < K; k++) {
        for (int l = 0; l < nl; l++) {
            ZK_CHECK_HIP(hipSetDevice(X.P[l]->device));
            hash(l, scratch[l] + k * piece, log_QG, log_K, k);
            snd[l] = scratch[l] + k * piece;
            rcv[l] = scratch[l] + 32 * Q + k * piece;
        }
        ZK_TRY(xchg_start(X, digests_name, A2A, snd, rcv, (size_t)32 << log_QGK, &h[k]));
    }
    for (int k = 0; k < K; k++) {
        ZK_TRY(xchg_wait(X, h[k]));
        for (int l = 0; l < nl; l++) {
            zk_prover *p = X.P[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            hipLaunchKernelGGL(k_sh_blk_merge, dim3(cdiv(Q / K / 2, 256)), dim3(256), 0, p->st,
                               (const uint8_t *)scratch[l] + 32 * Q + k * piece, X.G, log_QGK, k, nodes[l] + 32 * (Q / 2));
        }
    }
    std::vector<const void *> rs(nl);
    std::vector<void *> rr(nl);
    for (int l = 0; l < nl; l++) {
        zk_prover *p = X.P[l];
        ZK_CHECK_HIP(hipSetDevice(p->device));
        merkle_tree(p->st, nodes[l] + 32 * (Q / 2), Q / 2, nodes[l]);  // (Q >= G >= 2)
        rs[l] = nodes[l] + 32;
        rr[l] = p->sh_roots;
    }
    ZK_TRY(xchg(X, roots_name, AG, rs, rr, 32));
    std::vector<uint8_t> roots(32 * X.G);
    ZK_TRY(d2h_small(X.P[0], roots.data(), X.P[0]->sh_roots, roots.size()));
    ZK_TRY(d2h_flush(X.P[0]));
    T.top.assign(2 * X.G, {});
    for (int d = 0; d < X.G; d++) memcpy(T.top[X.G + d].data(), &roots[32 * d], 32);
    for (int k = X.G - 1; k >= 1; k--) {
        uint8_t buf[64];
        memcpy(buf, T.top[2 * k].data(), 32);
        memcpy(buf + 32, T.top[2 * k + 1].data(), 32);
        b3::hash_bytes(buf, 64, T.top[k].data());
    }
    memcpy(T.root, T.top[1].data(), 32);
    return ZK_OK;
}

int prove_sharded(Ctx &X, const uint8_t *trace, const zk_options *opt, const zk_pub_inputs *pub, uint8_t *proof_out,
                  size_t *proof_len, zk_record *rec) {
    const int G = X.G, Bl = X.Bl, log_n = X.log_n, C = X.C, nlp = (int)X.P.size();
    // FieldExtension: KX = 1 (None) or 2 (Quadratic, every E-valued buffer planar: plane stride Bl*n per rank)
    const int KX = (int)opt->field_extension, CK = C * KX;
    auto COMP = [&](zk_prover *p) { return KX == 2 ? p->x_comp : p->comp; };
    auto CTMP = [&](zk_prover *p) { return KX == 2 ? p->x_ctmp : p->ctmp; };
    auto CLDE = [&](zk_prover *p) { return KX == 2 ? p->x_clde : p->clde; };
    auto DEEP = [&](zk_prover *p) { return KX == 2 ? p->x_deep : p->deep; };
    auto FRI = [&](zk_prover *p) { return KX == 2 ? p->x_fri : p->fri; };
    const size_t n = X.n, N = 8 * n, CE = 8 * n;
    const uint32_t fold = opt->fri_folding;
    const size_t m = n / fold;          // FRI layer-0 positions per coset
    const int log_m = ilog2(m);
    const fe g = h_root_of_unity(log_n), three = fe_make(3);
    zk_prover *P0 = X.P[0];
    for (zk_prover *p : X.P) ZK_TRY(io_rewind(p));  // the pinned staging areas start over
    zk_record R;
    memset(&R, 0, sizeof R);
    R.trace_len = (uint32_t)n;
    R.lde_len = (uint32_t)N;
    R.width = W;
    R.num_ccols = (uint32_t)C;
    stage_begin(P0);
    stage_mark(P0, "start");
    Coin coin = seed_coin(n, opt, pub);

    // S2: the trace polynomials on every rank, then the local coset LDE and the distributed commitment.  Every trace
    // source splits the interpolation by column, round robin: in round k rank g interpolates column U[g + G k] and an
    // all-gather (in place when the round's columns are consecutive) fills the round's G columns on every rank, after
    // which every rank extends them over its cosets.  Round k's all-gather runs on the exchange stream while the
    // compute stream interpolates round k + 1 and extends round k - 1 (xchg_start / xchg_wait), so each rank computes
    // 1/G of the coefficients and the exchange hides under the coset LDEs.  U (the columns transformed) leaves out
    // what every rank forms from the last row alone (sparse columns, the AIR clock) or from per-program tables:
    //  * host trace: rank g uploads (copy stream) only its own columns, so each rank moves 1/G of the trace over PCIe;
    //    the previous sharded proof's column hints (sparse, clock, narrow) as the single-GPU host path (section 6c);
    //  * trace already in every rank's HBM (trace = NULL): each rank detects the sparse columns and the clock over its
    //    1/G of the rows, the flags are all-gathered (round 6: the interpolation was replicated before, 4.0 ms of
    //    every rank's time at 2^22);
    //  * zk_vm_prove_sharded: only the dynamic stack columns; the program-only columns from the preprocessed tables.
    const fe inv_n = h_inv(fe_make(n));
    const size_t col = n * sizeof(fe);
    // on an early error return, copies from the caller's host trace may still be in flight: the caller may free it
    // as soon as this returns (the rounds of a completed S2 have waited for every copy)
    struct CopyGuard {
        const std::vector<zk_prover *> &P;
        bool on;
        ~CopyGuard() {
            if (!on) return;
            for (zk_prover *p : P) {
                (void)hipSetDevice(p->device);
                upload_drain(p);
                // (and the kernels of a failed proof: the next proof's uploads into d_trace must not overtake them)
                (void)hipStreamSynchronize(p->st);
                if (p->cst) (void)hipStreamSynchronize(p->cst);
            }
        }
    } copy_guard{X.P, trace != nullptr};
    // host checks of the hinted columns (below): the tasks read the caller's trace, so every way out waits for them
    Latch checked, packed;
    std::unique_ptr<std::atomic<uint32_t>[]> bad(new std::atomic<uint32_t>[nlp]), pack_bad(new std::atomic<uint32_t>[nlp]);
    for (int l = 0; l < nlp; l++) {
        bad[l].store(0);
        pack_bad[l].store(0);
    }
    struct CheckWait {
        Latch &a, &b;
        ~CheckWait() {
            a.wait();
            b.wait();
        }
    } check_wait{checked, packed};
    int U[W], nU = 0;     // the columns interpolated, ascending
    uint32_t S = 0;       // sparse columns (zero but the last row): coefficients and LDE from the last row
    bool clk = false;       // the AIR clock (column 0 = 0 .. n-2 but the last row): from the identity column's tables
    fe lastv[W];          // the last row (host trace, device trace: read back with the flags)
    std::vector<SparseCols> spc(nlp);
    std::vector<const SparseCols *> spp(nlp, nullptr);
    std::vector<NarrowCols> nar(nlp);
    std::vector<uint32_t> went_packed(nlp, 0u);
    uint32_t N8 = 0, N32 = 0;
    zk_prover *H = X.P[0];
    if (trace) {
        // Column classes (round 4, as the single-GPU host path): the sparse columns (zero but the last row) and the AIR
        // clock (rows 0 .. n-2 = 0 .. n-2) that the previous sharded proof of this length, world and program found --
        // the same hints on every rank, learned from all-gathered flags -- are neither uploaded, interpolated nor
        // all-gathered: every rank forms their coefficients and local LDE from the last row (fills).  Each rank's host
        // threads check its 1/G row range of them; the flags are all-gathered with the hints of the next proof, and a
        // refuted hint voids the proof on every rank (prove_sharded_entry redoes it without hints).
        static const bool hints_on = [] {  // ZK_SHARD_HINTS=0: every column uploaded, interpolated and all-gathered
            const char *e = getenv("ZK_SHARD_HINTS");
            return !(e && !strcmp(e, "0"));
        }();
        // (keyed by length, world and program: column classes are a property of the program)
        const bool fresh = hints_on && X.hint_ok && sparse_on() && X.pl[0]->lagr && H->sh_hint_n == n && H->sh_hint_g == G &&
                           !memcmp(H->sh_hint_key, pub->program_hash, 32);
        S = fresh ? H->sh_sparse : 0u;
        clk = fresh && H->sh_clock && clock_on() && H->sh_clock_off_n != n && !(S & 1u);
        X.sh_clock = clk;
        const uint32_t derived = S | (clk ? 1u : 0u);
        N8 = fresh && narrow_on() ? H->sh_nw8 & ~derived : 0u;
        N32 = fresh && narrow_on() ? H->sh_nw32 & ~derived & ~N8 : 0u;
        for (int c = 0; c < W; c++)
            if (!((S >> c) & 1u) && !(clk && c == 0)) U[nU++] = c;
        static_assert((W + 1) / 2 <= ZK_UPLOAD_GROUPS_MAX, "one upload event per round at G = 2");
        for (int c = 0; c < W; c++) memcpy(&lastv[c], trace + (size_t)c * col + (n - 1) * sizeof(fe), sizeof(fe));
        for (int l = 0; l < nlp; l++) {
            ZK_CHECK_HIP(hipSetDevice(X.P[l]->device));
            ZK_TRY(sparse_begin(X.P[l], X.pl[l], &spc[l], &spp[l]));  // the flags the interpolation's pass 1 sets
            if (spp[l]) spc[l].wstride = W;
            if (clk) ZK_TRY(clock_tables(X.P[l], X.pl[l]));
        }
        if (S | (clk ? 1u : 0u)) {
            constexpr size_t R = (size_t)1 << 18;
            std::vector<std::pair<int, size_t>> tasks;  // (local rank, first row)
            for (int l = 0; l < nlp; l++) {
                const size_t r0 = n * (size_t)X.rank[l] / (size_t)G, r1 = std::min(n - 1, n * (size_t)(X.rank[l] + 1) / G);
                for (size_t t = r0; t < r1; t += R) tasks.push_back({l, t});
            }
            int nt = 0;
            for (int c = 0; c < W; c++) nt += ((S >> c) & 1u) || (clk && c == 0) ? 1 : 0;
            checked.reset(nt * (int)tasks.size());
            for (int c = 0; c < W; c++) {
                const bool sparse = (S >> c) & 1u, clock = clk && c == 0;
                if (!sparse && !clock) continue;
                const uint8_t *cp = trace + (size_t)c * col;
                for (const auto &tk : tasks) {
                    const int l = tk.first;
                    const size_t t0 = tk.second;
                    const size_t r1 = std::min(n - 1, std::min(n * (size_t)(X.rank[l] + 1) / G, t0 + R));
                    std::atomic<uint32_t> *b = &bad[l];
                    HostPool::get().submit([=, &checked] {
                        if (!(clock ? clock_rows(cp, t0, r1) : zero_rows(cp, t0, r1))) b->fetch_or(1u << c);
                        checked.count_down();
                    });
                }
            }
        }
        // narrow columns (8- or 32-bit before the last row): their owner's host threads pack rows 0 .. n-2 into its
        // pinned staging while the other columns go up; a column goes up packed (expanded on the device), or whole if a
        // value does not fit
        for (int l = 0; l < nlp; l++) {
            NarrowCols &nc = nar[l];
            nc.count = 0;
            size_t bytes = 0;
            for (int i = X.rank[l]; i < nU; i += G) {
                const int c = U[i];
                if (!(((N8 | N32) >> c) & 1u)) continue;
                nc.col[nc.count] = c;
                nc.width[nc.count] = ((N8 >> c) & 1u) ? 1 : 4;
                nc.off[nc.count] = bytes;
                nc.last[nc.count] = lastv[c];
                bytes += ((size_t)nc.width[nc.count] * n + 15) & ~(size_t)15;
                nc.count++;
            }
            zk_prover *p = X.P[l];
            if (nc.count && bytes > p->h_pack_cap) {  // (the previous proof's copies from it have drained: CopyGuard)
                if (p->h_pack) (void)hipHostFree(p->h_pack);
                p->h_pack = nullptr;
                p->h_pack_cap = 0;
                ZK_CHECK_HIP(hipHostMalloc((void **)&p->h_pack, bytes, hipHostMallocMapped | hipHostMallocCoherent));
                p->h_pack_cap = bytes;
            }
        }
        {
            constexpr size_t R = (size_t)1 << 18;
            const size_t per = (n - 1 + R - 1) / R;
            int total = 0;
            for (int l = 0; l < nlp; l++) total += nar[l].count * (int)per;
            packed.reset(total);
            for (int l = 0; l < nlp; l++)
                for (int k = 0; k < nar[l].count; k++)
                    for (size_t t = 0; t < per; t++) {
                        const size_t r0 = t * R, r1 = std::min(n - 1, r0 + R);
                        const uint8_t *cp = trace + (size_t)nar[l].col[k] * col;
                        uint8_t *dst = X.P[l]->h_pack + nar[l].off[k];
                        const int width = nar[l].width[k], c = nar[l].col[k];
                        std::atomic<uint32_t> *b = &pack_bad[l];
                        HostPool::get().submit([=, &packed] {
                            if (!pack_rows(cp, r0, r1, width, dst)) b->fetch_or(1u << c);
                            if (r1 == n - 1) memset(dst + (size_t)width * (n - 1), 0, width);  // (the last row's slot)
                            packed.count_down();
                        });
                    }
        }
    } else if (X.fixed) {
        // vm::prove: the dynamic stack columns only (12 .. 12 + md - 1); the program-only columns and the zero registers
        // from the per-program preprocessed columns of this rank's cosets (one streaming pass, after the rounds)
        for (int c = 12; c < 12 + X.fixed[0].md; c++) U[nU++] = c;
    } else {
        // every rank holds the whole trace: each detects the sparse columns and the clock over its 1/G of the rows
        // (whole 4096-row blocks; shorter traces: every row), the flags are all-gathered and OR-ed, and every rank reads
        // them back with the last row (one host round trip) to plan the rounds
        const size_t rr = n / (size_t)G;
        const bool row_split = rr % 4096 == 0;
        bool detect = true;
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            ZK_TRY(sparse_begin(p, X.pl[l], &spc[l], &spp[l]));
            if (!spp[l]) {
                detect = false;
                continue;
            }
            const size_t r0 = row_split ? rr * (size_t)X.rank[l] : 0, r1 = row_split ? r0 + rr : n;
            sparse_detect_rows(p->st, p->d_trace, n, 0, W, spc[l], r0, r1);
        }
        if (detect) {
            std::vector<const void *> fs(nlp);
            std::vector<void *> fr(nlp);
            for (int l = 0; l < nlp; l++) {
                fs[l] = X.P[l]->sp_nz;
                fr[l] = X.P[l]->sh_buf;
            }
            ZK_TRY(xchg(X, "column_flags", AG, fs, fr, 4 * W * sizeof(unsigned)));
            std::vector<unsigned> f((size_t)G * 4 * W);
            ZK_CHECK_HIP(hipSetDevice(P0->device));
            ZK_TRY(d2h_small(P0, f.data(), P0->sh_buf, f.size() * sizeof(unsigned)));
            ZK_TRY(d2h_small(P0, lastv, P0->sp_last, sizeof lastv));
            ZK_TRY(d2h_flush(P0));
            unsigned nz[4 * W] = {};
            for (int g = 0; g < G; g++)
                for (int c = 0; c < 4 * W; c++) nz[c] |= f[(size_t)g * 4 * W + c];
            for (int c = 0; c < W; c++)
                if (nz[c] == 0) S |= 1u << c;
            clk = clock_on() && !(S & 1u) && nz[3 * W] == 0 && spc[0].id_poly;
        }
        for (int c = 0; c < W; c++)
            if (!((S >> c) & 1u) && !(clk && c == 0)) U[nU++] = c;
        if (clk)
            for (int l = 0; l < nlp; l++) ZK_TRY(clock_tables(X.P[l], X.pl[l]));
    }
    // the narrow column k of local rank l, or -1
    auto narrow_of = [&](int l, int c) {
        for (int k = 0; k < nar[l].count; k++)
            if (nar[l].col[k] == c) return k;
        return -1;
    };
    auto upload = [&](int k) -> int {  // host trace: round k's column of every local rank onto its copy stream
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            const int i = X.rank[l] + G * k;
            ZK_CHECK_HIP(hipSetDevice(p->device));
            const int q = i < nU ? narrow_of(l, U[i]) : -1;
            if (q >= 0) packed.wait();  // (before the lock: the packing does not need it)
            std::lock_guard<std::mutex> lk(*p->up_mu);
            UploadEvent rec{p->ev_up[k], p->up};  // recorded on the error path too (CopyGuard drains it)
            if (q >= 0 && !((pack_bad[l].load() >> U[i]) & 1u)) {
                const size_t w = (size_t)nar[l].width[q] * n;
                ZK_CHECK_HIP(hipMemcpyAsync(reinterpret_cast<uint8_t *>(CLDE(p)) + nar[l].off[q],
                                            p->h_pack + nar[l].off[q], w, hipMemcpyHostToDevice, p->up));
                went_packed[l] |= 1u << U[i];
            } else if (i < nU) {
                ZK_CHECK_HIP(hipMemcpyAsync(p->d_trace + (size_t)U[i] * n, trace + (size_t)U[i] * col, col,
                                            hipMemcpyHostToDevice, p->up));
            }
            ZK_TRY(rec.record());
        }
        return ZK_OK;
    };
    // device-resident traces: the first `rep` columns of U are interpolated by every rank itself (no exchange), right
    // after rounds 0 and 1's all-gathers start, so they fill the time those take; the rest go round robin.  A host trace splits
    // every column: replicating one would make every rank upload it.
    int rep = 0;
    if (!trace) {
        // from the replayed schedules of 2^22 proofs (profiles/r06zc_split_sweep_2p22.json):
        // with two rounds in flight four columns hide rounds 0 and 1 at every world size (at G = 2 replicating every
        // column, the one-round-in-flight optimum, is 1.1 ms slower)
        const int dflt = 4;
        rep = std::min(nU, X.comm->split_rep >= 0 ? X.comm->split_rep : dflt);
    }
    const int nrep = rep;  // U[0 .. rep) replicated
    int *US = U + rep;     // the split columns
    const int nS = nU - rep;
    const int rounds = (nS + G - 1) / G;
    std::vector<XH> hr(std::max(rounds, 1));
    std::vector<char> inplace_r(std::max(rounds, 1));
    // a round whose columns are not consecutive is gathered into a staging area, alternating between two buffers
    // free until S3 / S4, so round k + 1's all-gather never overwrites what round k's copy-out still reads
    auto stage_of = [&](zk_prover *p, int k) { return (k & 1) ? p->comp : p->ctmp; };
    // in place when the round's columns are consecutive (the padding slots of a short last round then land on columns
    // nobody interpolates -- filled below -- or past W: p->polys holds 8 ceil(W / 8) columns)
    auto inplace_of = [&](int k) {
        const int i0 = G * k, real = std::min(G, nS - i0), first = US[i0];
        return US[i0 + real - 1] - first == real - 1 && first + G <= 8 * ((W + 7) / 8);
    };
    auto issue = [&](int k) -> int {  // interpolate this rank's column of round k, start the round's all-gather
        if (trace && k + 1 < rounds) ZK_TRY(upload(k + 1));
        const int i0 = G * k, real = std::min(G, nS - i0), first = US[i0];
        const bool inplace = inplace_of(k);
        inplace_r[k] = inplace;
        std::vector<const void *> snd(nlp);
        std::vector<void *> rcv(nlp);
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            const int i = i0 + X.rank[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            if (trace) {
                // (a device-side wait: a sharded rank's process holds one prover, so its compute, exchange and upload
                // streams have hardware queues of their own and the host never blocks on the link)
                ZK_CHECK_HIP(hipStreamWaitEvent(p->st, p->ev_up[k], 0));
                if (i < nS && ((went_packed[l] >> US[i]) & 1u)) {
                    const int q = narrow_of(l, US[i]);
                    NarrowCols one{};
                    one.count = 1;
                    one.col[0] = US[i];
                    one.width[0] = nar[l].width[q];
                    one.off[0] = nar[l].off[q];
                    one.last[0] = nar[l].last[q];
                    expand_narrow(p->st, reinterpret_cast<const uint8_t *>(CLDE(p)), one, n, p->d_trace);
                }
            }
            if (i < nS) {
                SparseCols g = spc[l];
                g.col0 = US[i];
                g.fused = true;
                ntt(p->st, X.pl[l]->Tn, p->d_trace + (size_t)US[i] * n, n, p->polys + (size_t)US[i] * n, n, 1, true, nullptr,
                    &inv_n, p->tmp, trace && spp[l] ? &g : nullptr);
            }
            snd[l] = inplace ? p->polys + (size_t)(first + X.rank[l]) * n : p->polys + (size_t)(i < nS ? US[i] : 0) * n;
            rcv[l] = inplace ? p->polys + (size_t)first * n : stage_of(p, k);
        }
        return xchg_start(X, "trace_coeffs", AG, snd, rcv, col, &hr[k]);
    };
    auto finish = [&](int k) -> int {  // wait for round k's coefficients, extend them over the local cosets
        ZK_TRY(xchg_wait(X, hr[k]));
        const int i0 = G * k, real = std::min(G, nS - i0);
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            if (!inplace_r[k])
                for (int g = 0; g < real; g++)
                    if (g != X.rank[l])
                        ZK_CHECK_HIP(hipMemcpyAsync(p->polys + (size_t)US[i0 + g] * n, stage_of(p, k) + (size_t)g * n, col,
                                                    hipMemcpyDeviceToDevice, p->st));
            for (int a = 0; a < real;) {
                int b = a + 1;
                while (b < real && US[i0 + b] == US[i0 + b - 1] + 1) b++;
                const int c0 = US[i0 + a];
                ntt_lde(p->st, X.pl[l]->Tn, X.pl[l]->ct, p->polys + (size_t)c0 * n, n, b - a, X.rank[l] * Bl, 1, Bl,
                        p->lde + (size_t)c0 * Bl * n, (size_t)Bl * n, n, p->tmp);
                a = b;
            }
        }
        return ZK_OK;
    };
    if (trace && rounds) ZK_TRY(upload(0));
    // two rounds in flight: rounds 0 and 1 go out before the replicated columns, and round k + 2 before round k's
    // extension when it is gathered in place (after it when staged: it reuses round k's staging buffer), so the link
    // always has the next round queued
    for (int k = 0; k < std::min(rounds, 2); k++) ZK_TRY(issue(k));
    if (nrep) {
        ZK_TRY(sched_entry(X, 'K', -1));
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            for (int a = 0; a < nrep;) {
                int b = a + 1;
                while (b < nrep && U[b] == U[b - 1] + 1) b++;
                const int c0 = U[a];
                ntt(p->st, X.pl[l]->Tn, p->d_trace + (size_t)c0 * n, n, p->polys + (size_t)c0 * n, n, b - a, true, nullptr,
                    &inv_n, p->tmp);
                ntt_lde(p->st, X.pl[l]->Tn, X.pl[l]->ct, p->polys + (size_t)c0 * n, n, b - a, X.rank[l] * Bl, 1, Bl,
                        p->lde + (size_t)c0 * Bl * n, (size_t)Bl * n, n, p->tmp);
                a = b;
            }
        }
    }
    for (int k = 0; k < rounds; k++) {
        const bool next = k + 2 < rounds, ahead = next && inplace_of(k + 2);
        if (ahead) ZK_TRY(issue(k + 2));
        ZK_TRY(finish(k));
        if (next && !ahead) ZK_TRY(issue(k + 2));
    }
    // the columns formed from the last row (after the last round: a short round's padding may have landed there)
    if (X.fixed) {
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            const FixedCols &fx = X.fixed[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            if (!p->fix_ws) ZK_CHECK_HIP(p->arena.alloc(&p->fix_ws, W));
            fe_ws ws[W];
            for (int c = 0; c < W; c++) ws[c] = make_fe_ws(fx.last[c]);
            ZK_TRY(h2d_small(p, p->fix_ws, ws, sizeof ws));
            fixed_axpy(p->st, fx, p->fix_ws, n, (size_t)Bl, p->polys, p->lde);
        }
    } else if (S | (clk ? 1u : 0u)) {
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            if (S) {
                if (trace) ZK_TRY(h2d_small(p, p->sp_last, lastv, sizeof lastv));  // (device traces: the detection's)
                for (int c = 0; c < W;) {
                    if (!((S >> c) & 1u)) {
                        c++;
                        continue;
                    }
                    int e = c + 1;
                    while (e < W && ((S >> e) & 1u)) e++;
                    SparseCols g = spc[l];
                    g.col0 = c;
                    g.fused = false;
                    g.all = true;  // fills only
                    ntt(p->st, X.pl[l]->Tn, p->polys + (size_t)c * n, n, p->polys + (size_t)c * n, n, e - c, true, nullptr,
                        &inv_n, p->tmp, &g);
                    ntt_lde(p->st, X.pl[l]->Tn, X.pl[l]->ct, p->polys + (size_t)c * n, n, e - c, X.rank[l] * Bl, 1, Bl,
                            p->lde + (size_t)c * Bl * n, (size_t)Bl * n, n, p->tmp, &g);
                    c = e;
                }
            }
            if (clk) {
                const fe_ws d = make_fe_ws(fe_sub(lastv[0], fe_make(n - 1)));
                const Plan *pl = X.pl[l];
                axpy_fill(p->st, pl->id_poly, pl->lagr, d, n, p->polys);
                for (int j = 0; j < Bl; j++) {
                    const size_t r = (size_t)X.rank[l] * Bl + j;
                    axpy_fill(p->st, pl->id_lde + pl->lde_slot((int)r) * n, pl->lagr_lde + pl->lde_slot((int)r) * n, d,
                              n, p->lde + (size_t)j * n);
                }
            }
        }
    }
    // host traces: the flags of the columns each rank interpolated (for the next proof's hints) and each rank's check
    // of the hinted ones, all-gathered: every rank then holds the same view
    if (trace && spp[0]) {
        checked.wait();
        std::vector<const void *> fs(nlp);
        std::vector<void *> fr(nlp);
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            const uint32_t b = bad[l].load();
            ZK_TRY(h2d_small(p, p->sp_nz + 3 * W + 1, &b, sizeof b));
            fs[l] = p->sp_nz;
            fr[l] = p->sh_buf;
        }
        ZK_TRY(xchg(X, "column_flags", AG, fs, fr, 4 * W * sizeof(unsigned)));
        std::vector<unsigned> f((size_t)G * 4 * W);
        ZK_TRY(d2h_small(P0, f.data(), P0->sh_buf, f.size() * sizeof(unsigned)));
        ZK_TRY(d2h_flush(P0));
        unsigned nz[3 * W] = {};
        uint32_t refuted = 0;
        for (int g = 0; g < G; g++) {
            for (int c = 0; c < 3 * W; c++) nz[c] |= f[(size_t)g * 4 * W + c];
            refuted |= f[(size_t)g * 4 * W + 3 * W + 1];
        }
        if (refuted) {
            X.sh_refuted = refuted;
            return ZK_SH_REDO;
        }
        // next proof: the columns found sparse (uploaded ones with no nonzero entry before the last row, and the
        // hinted ones, which the checks confirmed), narrow (8- / 32-bit before the last row), and the clock when
        // column 0 was found 32-bit (or was derived)
        uint32_t sp_next = S, w8 = 0, w32 = 0;
        for (int i = 0; i < nU; i++) {
            const int c = U[i];
            if (nz[c] == 0) sp_next |= 1u << c;
            else if (nz[W + c] == 0) w8 |= 1u << c;
            else if (nz[2 * W + c] == 0) w32 |= 1u << c;
        }
        const bool clk_next = clk || (!(sp_next & 1u) && (w32 & 1u));
        if (clk_next) w32 &= ~1u;
        for (zk_prover *p : X.P) {
            p->sh_sparse = sp_next;
            p->sh_nw8 = w8;
            p->sh_nw32 = w32;
            p->sh_clock = clk_next;
            p->sh_hint_n = n;
            p->sh_hint_g = G;
            memcpy(p->sh_hint_key, pub->program_hash, 32);
        }
    }
    stage_mark(P0, "trace_lde");
    std::vector<uint8_t *> scratch(nlp), nd(nlp);
    for (int l = 0; l < nlp; l++) {
        scratch[l] = X.P[l]->fri_dig;
        nd[l] = X.P[l]->nodes;
    }
    DistTree Ttrace;
    // the row hashes of local rank l's cosets, piece k (Bl = 1, 2, 4 -> its template instance)
    auto hash_rows = [&](int l, const fe *base, int ncols, uint8_t *blk, uint8_t *send, int log_QG, int log_K, int k) {
        const dim3 grid(cdiv(n >> log_K, 256));
        hipStream_t st = X.P[l]->st;
        if (Bl == 4) hipLaunchKernelGGL(k_sh_hash_rows_blk<4>, grid, dim3(256), 0, st, base, ncols, log_n, log_QG, log_K, k, blk, send);
        else if (Bl == 2) hipLaunchKernelGGL(k_sh_hash_rows_blk<2>, grid, dim3(256), 0, st, base, ncols, log_n, log_QG, log_K, k, blk, send);
        else hipLaunchKernelGGL(k_sh_hash_rows_blk<1>, grid, dim3(256), 0, st, base, ncols, log_n, log_QG, log_K, k, blk, send);
    };
    std::vector<uint8_t *> bk(nlp);
    for (int l = 0; l < nlp; l++) bk[l] = X.P[l]->sh_blk;
    ZK_TRY(dist_commit(X, Ttrace, N, [&](int l, uint8_t *send, int log_QG, int log_K, int k) {
        hash_rows(l, X.P[l]->lde, W, X.P[l]->sh_blk, send, log_QG, log_K, k);
    }, scratch, bk, nd, "trace_digests", "trace_roots"));
    memcpy(R.trace_root, Ttrace.root, 32);
    stage_mark(P0, "trace_commit");
    coin.reseed(R.trace_root);

    // S3: constraint evaluation over the local CE cosets (CE domain = LDE domain at blowup 8).  The assertion terms
    // are not evaluated per row: S4 adds their quotient in coefficient form, each rank over its n / G coefficient
    // slice (boundary_range_*; traces too short for whole ranges keep the per-row form).
    const bool bnd_split = (n / G) % ZK_DEEP_RANGE_QUANTUM == 0;
    AirConsts K, Kp[2];
    if (KX == 1) {
        draw_air_consts(coin, pub, n, K, R);
    } else {
        draw_air_consts_ext(coin, pub, n, Kp[0], Kp[1], R);
        K = Kp[0];
    }
    for (int l = 0; l < nlp; l++) {
        zk_prover *p = X.P[l];
        Plan *pl = X.pl[l];
        ZK_CHECK_HIP(hipSetDevice(p->device));
        // divisor tables of the local CE cosets (3 planes of Bl*n): they depend on n and the cosets only, so the plan
        // keeps them for the rank's next proofs (round 6: 0.26 ms per rank and proof at G = 8, 2^22)
        const int r0 = X.rank[l] * Bl;
        if (!pl->sh_divs || pl->sh_divs_r0 != r0 || pl->sh_divs_cos != Bl) {
            if (pl->sh_divs && pl->sh_divs_cos < Bl) pl->sh_divs = nullptr;  // (a full prover serving a smaller world)
            if (!pl->sh_divs) ZK_CHECK_HIP(p->arena.alloc(&pl->sh_divs, (size_t)3 * Bl * n));
            fe xr[8];
            for (int j = 0; j < Bl; j++) xr[j] = K.xr[r0 + j];
            ZK_TRY(h2d_small(p, p->sh_xr, xr, Bl * sizeof(fe)));
            Fe8 zloc{};
            for (int j = 0; j < Bl; j++) zloc.v[j] = K.inv_zn[r0 + j];
            divisor_tables(p->st, pl->Tn, p->sh_xr, ilog2(Bl), log_n, K.g_last1, K.g_last2, zloc, pl->sh_divs);
            pl->sh_divs_r0 = r0;
            pl->sh_divs_cos = Bl;
        }
        if (KX == 1) ZK_TRY(h2d_small(p, p->air_consts, &K, sizeof K));
        else ZK_TRY(h2d_small(p, p->x_air, Kp, sizeof Kp));
    }

    // S3 + S4's first step, coset by coset (round 6): evaluate local coset j, inverse-transform it (KX planes), pack
    // its coefficient slices [d][plane][k'] and start its all-to-all, which then runs under coset j + 1's evaluation
    // instead of after the last one.  Piece j lands in the receive area [j][s][plane][k'] (after the KX*Bl*n
    // evaluations in COMP); the NTT scratch and the send areas are in p->tmp.
    const size_t kg = n / G;
    const size_t recv0 = (size_t)KX * Bl * n;  // the receive area's offset in COMP
    std::vector<XH> hs(Bl);
    for (int j = 0; j < Bl; j++) {
        std::vector<const void *> snd(nlp);
        std::vector<void *> rcv(nlp);
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            Plan *pl = X.pl[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            const EvalMap em{1, X.rank[l] * Bl + j, 1, 0, Bl, (size_t)Bl * n};
            if (KX == 1)
                ZK_CHECK_HIP(eval_constraints_mapped(p->st, p->lde + (size_t)j * n, log_n, em, pl->periodic,
                                                     pl->sh_divs + (size_t)j * n, (const AirConsts *)p->air_consts,
                                                     p->comp + (size_t)j * n, !bnd_split));
            else
                ZK_CHECK_HIP(eval_constraints_ext_mapped(p->st, p->lde + (size_t)j * n, log_n, em, pl->periodic,
                                                         pl->sh_divs + (size_t)j * n, (const AirConsts *)p->x_air,
                                                         (size_t)Bl * n, p->x_comp + (size_t)j * n, !bnd_split));
            fe *scr = p->tmp, *send = scr + (size_t)KX * n * (1 + j);
            ntt(p->st, pl->Tn, COMP(p) + (size_t)j * n, (size_t)Bl * n, CTMP(p) + (size_t)j * n, (size_t)Bl * n, KX, true,
                nullptr, nullptr, scr);
            hipLaunchKernelGGL(k_sh_pack_coset, dim3(cdiv((size_t)KX * n, 256)), dim3(256), 0, p->st,
                               (const fe *)CTMP(p) + (size_t)j * n, (size_t)Bl * n, log_n, KX, ilog2(kg), send);
            snd[l] = send;
            rcv[l] = COMP(p) + recv0 + (size_t)j * KX * n;
        }
        ZK_TRY(xchg_start(X, "comp_slices", A2A, snd, rcv, (size_t)KX * kg * sizeof(fe), &hs[j]));
    }
    stage_mark(P0, "constraints");

    // S4: composition polynomial: the cross-coset step on this rank's slice, all-gather of the C columns; then local
    // coset LDE + commitment
    XH hdeg;  // the degree flags' all-gather (read once the composition is committed)
    {
        // (the first plane's assertion quotient reads only the trace coefficients: it runs under the all-to-all, and
        // its range sums' all-gather follows the all-to-all's pieces on the exchange stream)
        std::vector<const void *> bnd0(nlp);
        std::vector<void *> bsum(nlp);
        XH hb0;
        for (int l = 0; bnd_split && l < nlp; l++) {
            zk_prover *p = X.P[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            bnd0[l] = boundary_range_begin(p->st, p->polys, log_n, KX == 1 ? K : Kp[0], K.g_last2, p->dscratch,
                                           (size_t)X.rank[l] * kg, kg);
            bsum[l] = p->sh_buf;
        }
        if (bnd_split) ZK_TRY(xchg_start(X, "bnd_totals", AG, bnd0, bsum, 2 * sizeof(fe), &hb0));
        for (XH &h : hs) ZK_TRY(xchg_wait(X, h));
        const fe scale = h_inv(fe_make(CE)), w8inv = h_inv(h_root_of_unity(3)), inv3n = h_inv(h_pow(three, n));
        std::vector<const void *> fs(nlp);
        std::vector<void *> fr(nlp);
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            ZK_CHECK_HIP(hipMemsetAsync(p->flag, 0, 4, p->st));
            for (int pln = 0; pln < KX; pln++) {  // base column (c, pln) of E column c -> CTMP slice c*KX + pln
                CrossMap cm;
                for (int r = 0; r < 8; r++)  // global coset r = s Bl + j: piece j, source s
                    cm.c[r] = COMP(p) + recv0 + ((size_t)(r % Bl) * G * KX + (size_t)(r / Bl) * KX + pln) * kg;
                cm.k0 = (size_t)X.rank[l] * kg;
                cm.kcount = kg;
                cm.pstride = (size_t)KX * kg;
                comp_cross_mapped(p->st, cm, X.pl[l]->Tce, X.pl[l]->inv3, scale, w8inv, inv3n, C, CTMP(p) + pln * kg,
                                  p->flag);
            }
            fs[l] = p->flag;
            fr[l] = p->sh_flags;
        }
        // the column polynomials: one all-gather per column, started in order on the exchange stream (they run back to
        // back); the coset LDE of a group of columns starts as soon as the group has arrived, so the later columns'
        // all-gathers run under the earlier columns' LDEs.  Over F the columns after column 0 go out before its
        // assertion quotient is added (over E the second plane's range sums would queue behind them).
        std::vector<XH> hc(CK);
        auto start_columns = [&](int c0, int c1) -> int {
            for (int c = c0; c < c1; c++) {
                std::vector<const void *> s2(nlp);
                std::vector<void *> r2(nlp);
                for (int l = 0; l < nlp; l++) {
                    s2[l] = CTMP(X.P[l]) + c * kg;
                    r2[l] = X.P[l]->cpolys + (size_t)c * n;
                }
                ZK_TRY(xchg_start(X, "comp_columns", AG, s2, r2, kg * sizeof(fe), &hc[c]));
            }
            return ZK_OK;
        };
        const int early = KX == 1 ? 1 : CK;  // columns [early, CK) start before the quotient
        if (early < CK) ZK_TRY(start_columns(early, CK));
        // assertion quotient over this rank's slice of composition column 0 (plane by plane: the division scratch is
        // shared); the range sums are all-gathered and each rank adds the later ranks' as its carry
        for (int pln = 0; bnd_split && pln < KX; pln++) {
            const AirConsts &Kb = KX == 1 ? K : Kp[pln];
            if (pln == 0) {
                ZK_TRY(xchg_wait(X, hb0));
            } else {
                std::vector<const void *> s2(nlp);
                for (int l = 0; l < nlp; l++) {
                    zk_prover *p = X.P[l];
                    ZK_CHECK_HIP(hipSetDevice(p->device));
                    s2[l] = boundary_range_begin(p->st, p->polys, log_n, Kb, K.g_last2, p->dscratch,
                                                 (size_t)X.rank[l] * kg, kg);
                }
                ZK_TRY(xchg(X, "bnd_totals", AG, s2, bsum, 2 * sizeof(fe)));
            }
            for (int l = 0; l < nlp; l++) {
                zk_prover *p = X.P[l];
                ZK_CHECK_HIP(hipSetDevice(p->device));
                hipLaunchKernelGGL(k_sh_suffix_carry, dim3(1), dim3(64), 0, p->st, p->sh_buf, G, X.rank[l], 2, p->ood);
                const size_t k0 = (size_t)X.rank[l] * kg;
                boundary_range_end(p->st, log_n, K.g_last2, p->dscratch, k0, kg, p->ood, CTMP(p) + pln * kg - k0, p->flag);
            }
        }
        ZK_TRY(start_columns(0, early));
        ZK_TRY(xchg_start(X, "degree_flags", AG, fs, fr, sizeof(unsigned), &hdeg));
        // groups hold >= 2^22 LDE points per launch, in the order the columns went out
        const int grp = (int)std::max<size_t>(1, ((size_t)1 << 22) / ((size_t)Bl * n));
        auto extend = [&](int a, int b) -> int {
            for (int c0 = a; c0 < b; c0 += grp) {
                const int c1 = std::min(b, c0 + grp);
                for (int c = c0; c < c1; c++) ZK_TRY(xchg_wait(X, hc[c]));
                for (int l = 0; l < nlp; l++) {
                    zk_prover *p = X.P[l];
                    ZK_CHECK_HIP(hipSetDevice(p->device));
                    ntt_lde(p->st, X.pl[l]->Tn, X.pl[l]->ct, p->cpolys + (size_t)c0 * n, n, c1 - c0, X.rank[l] * Bl, 1,
                            Bl, CLDE(p) + (size_t)c0 * Bl * n, (size_t)Bl * n, n, p->tmp);
                }
            }
            return ZK_OK;
        };
        ZK_TRY(extend(early, CK));
        ZK_TRY(extend(0, early));
    }
    for (int l = 0; l < nlp; l++) nd[l] = X.P[l]->cnodes;
    DistTree Tcomp;
    for (int l = 0; l < nlp; l++) bk[l] = X.P[l]->sh_cblk;
    ZK_TRY(dist_commit(X, Tcomp, N, [&](int l, uint8_t *send, int log_QG, int log_K, int k) {
        hash_rows(l, CLDE(X.P[l]), CK, X.P[l]->sh_cblk, send, log_QG, log_K, k);
    }, scratch, bk, nd, "comp_digests", "comp_roots"));
    memcpy(R.constraint_root, Tcomp.root, 32);
    stage_mark(P0, "composition");
    unsigned degree_flag = 0;
    {
        ZK_TRY(xchg_wait(X, hdeg));
        std::vector<unsigned> f(G);
        ZK_TRY(d2h_small(P0, f.data(), P0->sh_flags, G * sizeof(unsigned)));
        ZK_TRY(d2h_flush(P0));
        for (unsigned v : f) degree_flag |= v;
    }
    coin.reseed(R.constraint_root);

    // DEEP split by coefficient range (n / G per rank, whole phase-3 chunks): begin(p, k0) -> device totals (2 KX
    // elements), end(p, k0, ext) -> the coefficient buffer (KX planes of n); `upload` stages the DEEP constants
    const size_t nr = n / G;
    const bool deep_split = nr % ZK_DEEP_RANGE_QUANTUM == 0;
    auto deep_split_ranges = [&](int kx, auto begin, auto end, auto upload, std::vector<const fe *> &Dk) -> int {
        const int nc = 2 * kx;
        std::vector<const void *> snd(nlp);
        std::vector<void *> rcv(nlp);
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            ZK_TRY(upload(p));
            snd[l] = begin(p, (size_t)X.rank[l] * nr);
            rcv[l] = p->sh_buf;
        }
        ZK_TRY(xchg(X, "deep_totals", AG, snd, rcv, (size_t)nc * sizeof(fe)));
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            hipLaunchKernelGGL(k_sh_suffix_carry, dim3(1), dim3(64), 0, p->st, p->sh_buf, G, X.rank[l], nc, p->ood);
            Dk[l] = end(p, (size_t)X.rank[l] * nr, p->ood);
        }
        XH hp[2];  // (both planes' all-gathers go out before either is waited for)
        for (int plane = 0; plane < kx; plane++) {
            for (int l = 0; l < nlp; l++) {
                snd[l] = Dk[l] + (size_t)plane * n + (size_t)X.rank[l] * nr;
                rcv[l] = (void *)(Dk[l] + (size_t)plane * n);
            }
            ZK_TRY(xchg_start(X, "deep_slices", AG, snd, rcv, nr * sizeof(fe), &hp[plane]));
        }
        for (int plane = 0; plane < kx; plane++) ZK_TRY(xchg_wait(X, hp[plane]));
        return ZK_OK;
    };

    // S5: OOD frame -- every rank evaluates its 1/G of the coefficient range of the (replicated) polynomials, the
    // partial sums are all-gathered and added on the host -- then DEEP over the local cosets
    std::vector<fe> h;  // the OOD frame, flattened (k base elements per E value)
    // nv values per rank (ood_eval / ood_eval_ext output); the frame value v is sum over ranks of part[rank][v]
    auto ood_parts = [&](int nv, auto launch, std::vector<fe> &sum) -> int {
        std::vector<const void *> snd(nlp);
        std::vector<void *> rcv(nlp);
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            launch(p, X.rank[l]);
            snd[l] = p->ood;
            rcv[l] = p->sh_buf;
        }
        ZK_TRY(xchg(X, "ood_parts", AG, snd, rcv, (size_t)nv * sizeof(fe)));
        std::vector<fe> parts((size_t)G * nv);
        ZK_CHECK_HIP(hipSetDevice(P0->device));
        ZK_TRY(d2h_small(P0, parts.data(), P0->sh_buf, parts.size() * sizeof(fe)));
        ZK_TRY(d2h_flush(P0));
        sum.assign(nv, fe_zero());
        for (int d = 0; d < G; d++)
            for (int v = 0; v < nv; v++) sum[v] = fe_add(sum[v], parts[(size_t)d * nv + v]);
        return ZK_OK;
    };
    if (KX == 1) {
        const fe z = coin.draw(), zg = fe_mul(z, g);
        fe_to_bytes(z, R.z);
        ZK_TRY(ood_parts(2 * W + C, [&](zk_prover *p, int rank) {
            ood_eval(p->st, p->polys, W, p->cpolys, C, log_n, z, zg, p->ood_tab, p->partials, p->ood, rank, G);
        }, h));
        ood_reseed(coin, h.data(), C, R);
        stage_mark(P0, "ood");
        const DeepConsts D = draw_deep_consts(coin, h.data(), C, z, zg, R);
        std::vector<const fe *> Dk(nlp);
        if (deep_split) {
            // DEEP as an exact polynomial (kernels.hip), split by coefficient range: each rank combines and divides
            // its n / G coefficients, the ranges' totals are all-gathered for the suffix carries, and the quotient
            // slices are all-gathered (in place) before every rank extends it over its cosets
            ZK_TRY(deep_split_ranges(1, [&](zk_prover *p, size_t k0) {
                return deep_range_begin(p->st, p->polys, p->cpolys, C, log_n, p->deep_consts, z, zg, p->dscratch, k0, nr);
            }, [&](zk_prover *p, size_t k0, const fe *ext) {
                return deep_range_end(p->st, log_n, z, zg, p->dscratch, k0, nr, ext);
            }, [&](zk_prover *p) { return h2d_small(p, p->deep_consts, &D, sizeof D); }, Dk));
        } else {
            for (int l = 0; l < nlp; l++) {
                zk_prover *p = X.P[l];
                ZK_CHECK_HIP(hipSetDevice(p->device));
                ZK_TRY(h2d_small(p, p->deep_consts, &D, sizeof D));
                Dk[l] = deep_poly(p->st, p->polys, p->cpolys, C, log_n, p->deep_consts, z, zg, p->dscratch);
            }
        }
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            Plan *pl = X.pl[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            lde_cosets(p->st, pl->Tn, pl->ct, Dk[l], n, X.rank[l] * Bl, 1, Bl, p->deep, p->tmp);  // local cosets g Bl + j
        }
    } else {
        const fe2 z = coin.draw_ext(2), zg = fe2_mulb(z, g);
        fe_to_bytes(z.a, R.z);
        const int np = 2 * W + CK;
        std::vector<fe> hv;
        ZK_TRY(ood_parts(2 * np, [&](zk_prover *p, int rank) {
            ood_eval_ext(p->st, p->polys, W, p->cpolys, CK, log_n, z, zg, p->x_tab, p->x_partials, p->ood, rank, G);
        }, hv));
        std::vector<fe2> e;
        ood_reseed_ext(coin, hv, C, R, e, h);
        stage_mark(P0, "ood");
        const DeepConstsE D = draw_deep_consts_ext(coin, e, C, z, zg, R);
        std::vector<const fe *> Dk(nlp);
        if (deep_split) {
            ZK_TRY(deep_split_ranges(2, [&](zk_prover *p, size_t k0) {
                return deep_range_begin_ext(p->st, p->polys, p->cpolys, C, log_n, p->x_deep_consts, z, zg, p->x_dscratch,
                                            k0, nr);
            }, [&](zk_prover *p, size_t k0, const fe *ext) {
                return deep_range_end_ext(p->st, log_n, z, zg, p->x_dscratch, k0, nr, ext);
            }, [&](zk_prover *p) { return h2d_small(p, p->x_deep_consts, &D, sizeof D); }, Dk));
        } else {
            for (int l = 0; l < nlp; l++) {
                zk_prover *p = X.P[l];
                ZK_CHECK_HIP(hipSetDevice(p->device));
                ZK_TRY(h2d_small(p, p->x_deep_consts, &D, sizeof D));
                Dk[l] = deep_poly_ext(p->st, p->polys, p->cpolys, C, log_n, p->x_deep_consts, z, zg, p->x_dscratch);
            }
        }
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            Plan *pl = X.pl[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            for (int plane = 0; plane < 2; plane++)  // planar per rank: plane stride Bl * n
                lde_cosets(p->st, pl->Tn, pl->ct, Dk[l] + plane * n, n, X.rank[l] * Bl, 1, Bl,
                           p->x_deep + (size_t)plane * Bl * n, p->tmp);
        }
    }
    stage_mark(P0, "deep");

    // S6: FRI.  Layer 0 is sharded (its fold rows stay in one coset), and so is layer 1 when a layer follows it and
    // every rank holds enough of its rows; the next layer is all-gathered and the remaining layers run on local rank 0
    // of every process.
    const int nl = fri_num_layers(N, opt);
    if (nl > ZK_MAX_FRI_LAYERS) ZK_FAIL(ZK_ERR_INVALID_ARG, "too many FRI layers");
    R.num_fri_layers = (uint32_t)nl;
    std::vector<uint8_t *> f0n(nlp);  // the layer-0 tree's subtree heap (m nodes) in the NTT scratch
    const size_t rows0 = N / fold;  // layer-0 Merkle leaves
    std::vector<const fe *> layer_vals(nl + 1);
    // layer 1 committed and folded on every rank (sh1) and then layer lg = 2 all-gathered, else layer lg = 1; the
    // gathered layer's storage: natural (lbg 0) or coset-major over 8 cosets (3; FriLayout)
    const size_t m1 = m / fold;
    bool sh1 = false;
    int lg = 1, lbg = 0;
    DistTree Tfri1;
    std::vector<uint8_t *> f1n(nlp);
    std::vector<uint8_t *> layer_leaves(nl), layer_nodes(nl);
    std::vector<size_t> layer_len(nl + 1);
    std::vector<fe> rem_flat;
    layer_len[0] = N;
    DistTree Tfri0;
    auto remainder = [&](std::vector<fe> &rv) -> int {  // rv: KX planes of the last layer
        if (KX == 1) return remainder_step(rv, 8, coin, R, degree_flag);
        return remainder_step_ext(rv, 8, coin, R, degree_flag, rem_flat);
    };
    if (nl == 0) {
        // no folding: the remainder is the whole DEEP layer, all-gathered into natural order per plane
        std::vector<const void *> snd(nlp);
        std::vector<void *> rcv(nlp);
        for (int l = 0; l < nlp; l++) {
            snd[l] = DEEP(X.P[l]);
            rcv[l] = COMP(X.P[l]);
        }
        ZK_TRY(xchg(X, "remainder_layer", AG, snd, rcv, (size_t)KX * Bl * n * sizeof(fe)));
        ZK_TRY(lead_segment(X));
        ZK_CHECK_HIP(hipSetDevice(P0->device));
        for (int pln = 0; pln < KX; pln++)
            hipLaunchKernelGGL(k_sh_permute, dim3(cdiv(N, 256)), dim3(256), 0, P0->st,
                               (const uint8_t *)(COMP(P0) + (size_t)pln * Bl * n), G, Bl, log_n, 16,
                               (size_t)KX * Bl * n, (uint8_t *)(FRI(P0) + pln * N));
        std::vector<fe> rv(KX * N);
        ZK_TRY(d2h_small(P0, rv.data(), FRI(P0), rv.size() * sizeof(fe)));
        ZK_TRY(d2h_flush(P0));
        ZK_TRY(remainder(rv));
    } else {
        for (int l = 0; l < nlp; l++) {
            f0n[l] = (uint8_t *)X.P[l]->tmp;
            bk[l] = X.P[l]->sh_fblk;
        }
        ZK_TRY(dist_commit(X, Tfri0, rows0, [&](int l, uint8_t *send, int log_QG, int log_K, int k) {
            zk_prover *p = X.P[l];
            uint8_t *b = p->sh_fblk;
            const int f = (int)fold;
            const fe *d = KX == 1 ? p->deep : p->x_deep;
            if (Bl == 4) launch_fri0_blk<4>(p->st, KX, d, log_n, f, log_m, log_QG, log_K, k, b, send);
            else if (Bl == 2) launch_fri0_blk<2>(p->st, KX, d, log_n, f, log_m, log_QG, log_K, k, b, send);
            else launch_fri0_blk<1>(p->st, KX, d, log_n, f, log_m, log_QG, log_K, k, b, send);
        }, scratch, bk, f0n, "fri0_digests", "fri0_roots", false));
        memcpy(R.fri_roots[0], Tfri0.root, 32);
        coin.reseed(R.fri_roots[0]);
        // alpha of `layer` from the host coin, into every local rank's fold constants
        auto draw_fold = [&](int layer) -> int {
            FoldConsts F;
            FoldConstsE FE;
            if (KX == 1) {
                const fe alpha = coin.draw();
                fe_to_bytes(alpha, R.fri_alphas[layer]);
                F = fold_consts(alpha, fold);
            } else {
                const fe2 alpha = coin.draw_ext(2);
                fe_to_bytes(alpha.a, R.fri_alphas[layer]);
                FE = fold_consts_ext(alpha, fold);
            }
            for (int l = 0; l < nlp; l++) {
                zk_prover *p = X.P[l];
                ZK_CHECK_HIP(hipSetDevice(p->device));
                if (KX == 1) ZK_TRY(h2d_small(p, p->fold_consts, &F, sizeof F));
                else ZK_TRY(h2d_small(p, p->x_fold_consts, &FE, sizeof FE));
            }
            return ZK_OK;
        };
        ZK_TRY(draw_fold(0));
        for (int l = 0; l < nlp; l++) {  // layer 0 -> this rank's layer-1 values [plane][j][q0] in CTMP
            zk_prover *p = X.P[l];
            ZK_CHECK_HIP(hipSetDevice(p->device));
            sh_fri_fold0(p->st, KX, (int)fold, DEEP(p), log_n, Bl, X.rank[l], log_m,
                         KX == 1 ? (const void *)p->fold_consts : (const void *)p->x_fold_consts, X.pl[l]->TN.inv_lo,
                         X.pl[l]->TN.inv_hi, 1, CTMP(p));
        }
        // Layer 1 (round 6): with a layer after it and enough rows per rank it is committed and folded on every rank over
        // its own cosets, as layer 0 (block ownership keeps its leaves and fold rows local), and layer 2 is all-gathered
        // instead of layer 1; the lead rank runs the layers after the gathered one.
        sh1 = nl >= 2 && m1 >= 8 * (size_t)G;
        lg = sh1 ? 2 : 1;
        const size_t mg = sh1 ? m1 : m, Lg = 8 * mg;  // the gathered layer: positions per coset, length
        if (sh1) {
            for (int l = 0; l < nlp; l++) {
                f1n[l] = f0n[l] + 32 * m;  // (after the layer-0 subtree's m nodes)
                bk[l] = X.P[l]->sh_f1blk;
            }
            const int log_m1 = ilog2(m1);
            ZK_TRY(dist_commit(X, Tfri1, rows0 / fold, [&](int l, uint8_t *send, int log_QG, int log_K, int k) {
                zk_prover *p = X.P[l];
                uint8_t *b = p->sh_f1blk;
                const int f = (int)fold;
                if (Bl == 4) launch_fri0_blk<4>(p->st, KX, CTMP(p), log_m, f, log_m1, log_QG, log_K, k, b, send);
                else if (Bl == 2) launch_fri0_blk<2>(p->st, KX, CTMP(p), log_m, f, log_m1, log_QG, log_K, k, b, send);
                else launch_fri0_blk<1>(p->st, KX, CTMP(p), log_m, f, log_m1, log_QG, log_K, k, b, send);
            }, scratch, bk, f1n, "fri1_digests", "fri1_roots", false));
            memcpy(R.fri_roots[1], Tfri1.root, 32);
            coin.reseed(R.fri_roots[1]);
            ZK_TRY(draw_fold(1));
            for (int l = 0; l < nlp; l++) {  // layer 1 -> this rank's layer-2 values in COMP (N / fold: wstride fold)
                zk_prover *p = X.P[l];
                ZK_CHECK_HIP(hipSetDevice(p->device));
                sh_fri_fold0(p->st, KX, (int)fold, CTMP(p), log_m, Bl, X.rank[l], log_m1,
                             KX == 1 ? (const void *)p->fold_consts : (const void *)p->x_fold_consts, X.pl[l]->TN.inv_lo,
                             X.pl[l]->TN.inv_hi, fold, COMP(p));
            }
        }
        {
            // the gathered layer into the lead's FRI buffer: base field with layers after it, in place (chunk [s][j] is
            // coset s Bl + j: the layer arrives coset-major, which the layer kernels read through FriLayout); else through
            // a staging area, permuted into natural order per plane (over E each source's chunk holds both planes, and a
            // last layer goes to the host in natural order)
            const bool inplace = KX == 1 && nl > lg;
            std::vector<const void *> snd(nlp);
            std::vector<void *> rcv(nlp);
            for (int l = 0; l < nlp; l++) {
                zk_prover *p = X.P[l];
                snd[l] = sh1 ? COMP(p) : CTMP(p);
                rcv[l] = inplace ? FRI(p) : sh1 ? FRI(p) + KX * Lg : COMP(p);
            }
            ZK_TRY(xchg(X, sh1 ? "fri_layer2" : "fri_layer1", AG, snd, rcv, (size_t)KX * Bl * mg * sizeof(fe)));
            ZK_TRY(lead_segment(X));  // from here the FRI layers after it and the queries run on the lead rank alone
            ZK_CHECK_HIP(hipSetDevice(P0->device));
            const fe *stage = sh1 ? FRI(P0) + KX * Lg : COMP(P0);
            for (int pln = 0; !inplace && pln < KX; pln++)
                hipLaunchKernelGGL(k_sh_permute, dim3(cdiv(Lg, 256)), dim3(256), 0, P0->st,
                                   (const uint8_t *)(stage + (size_t)pln * Bl * mg), G, Bl, ilog2(mg), 16,
                                   (size_t)KX * Bl * mg, (uint8_t *)(FRI(P0) + pln * Lg));
            lbg = inplace ? 3 : 0;
        }
        layer_len[1] = rows0;
        layer_vals[lg] = FRI(P0);
        layer_len[lg] = Lg;
        {
            // the lead's layers: their coins run on the device as in the single-GPU path (fri_coin_launch: no host round
            // trip per layer), the host replays the transcript after one flush
            fe *next = FRI(P0) + KX * Lg;
            uint8_t *dig = P0->fri_dig;  // the all-to-all scratch is free once layers 0 (and 1) are committed
            fe *alpha_dev = nullptr;
            if (KX == 1) {
                const FoldConsts F = fold_consts(fe_zero(), fold);
                ZK_TRY(h2d_small(P0, P0->fold_consts, &F, sizeof F));
                alpha_dev = &((FoldConsts *)P0->fold_consts)->alpha;
            } else {
                const FoldConstsE F = fold_consts_ext(fe2_zero(), fold);
                ZK_TRY(h2d_small(P0, P0->x_fold_consts, &F, sizeof F));
                alpha_dev = &((FoldConstsE *)P0->x_fold_consts)->alpha.a;
            }
            ZK_TRY(h2d_small(P0, P0->fri_seed, coin.seed, 32));  // (the next reseed restarts the counter)
            for (int l = lg; l < nl; l++) {
                const size_t L = layer_len[l], rows = L / fold;
                layer_leaves[l] = dig;
                layer_nodes[l] = dig + 32 * rows;
                dig += 64 * rows;
                const int lb = l == lg ? lbg : 0;  // the gathered layer as it arrived
                if (KX == 1) commit_fri_layer(P0->st, layer_vals[l], L, (int)fold, layer_leaves[l], layer_nodes[l], lb);
                else commit_fri_layer_ext(P0->st, layer_vals[l], L, (int)fold, layer_leaves[l], layer_nodes[l], lb);
                fri_coin_launch(P0->st, (uint32_t *)P0->fri_seed, layer_nodes[l] + 32, KX, alpha_dev, P0->fri_alphas + 2 * l);
                if (KX == 1) fri_fold_launch(P0->st, layer_vals[l], L, (int)fold, P0->fold_consts, X.pl[0]->TN, N / L, next, lb);
                else fri_fold_ext_launch(P0->st, layer_vals[l], L, (int)fold, P0->x_fold_consts, X.pl[0]->TN, N / L, next, lb);
                layer_vals[l + 1] = next;
                layer_len[l + 1] = rows;
                next += KX * rows;
            }
            // one round trip: roots and device alphas of the lead's layers, the last layer
            std::vector<fe> rv(KX * layer_len[nl]), dalpha(2 * nl);
            for (int l = lg; l < nl; l++) ZK_TRY(d2h_small(P0, R.fri_roots[l], layer_nodes[l] + 32, 32));
            if (nl > lg)
                ZK_TRY(d2h_small(P0, dalpha.data() + 2 * lg, P0->fri_alphas + 2 * lg, 2 * (nl - lg) * sizeof(fe)));
            ZK_TRY(d2h_small(P0, rv.data(), layer_vals[nl], rv.size() * sizeof(fe)));
            ZK_TRY(d2h_flush(P0));
            for (int l = lg; l < nl; l++) {  // host replay of the same transcript
                coin.reseed(R.fri_roots[l]);
                const fe2 alpha = KX == 1 ? fe2{coin.draw(), fe_zero()} : coin.draw_ext(2);
                fe_to_bytes(alpha.a, R.fri_alphas[l]);
                if (!fe_eq(alpha.a, dalpha[2 * l]) || (KX == 2 && !fe_eq(alpha.b, dalpha[2 * l + 1])))
                    ZK_FAIL(ZK_ERR_DEVICE, "device FRI transcript diverged from the host transcript");
            }
            ZK_TRY(remainder(rv));
        }
    }
    stage_mark(P0, "fri");

    // S7 / S8: positions, then every rank gathers the chunks it owns; all-gather; the host combines
    std::vector<uint64_t> pos;
    ZK_TRY(grind_and_positions(P0, coin, opt, N, R, pos));
    const size_t nu = pos.size();
    const auto fri_pos = fri_fold_positions(pos, N, fold, nl);
    // (the openings, their plans and the request list keep their storage across proofs: this host work sits on every
    // rank's critical path, in the lead rank's segment, where fresh allocations cost page faults)
    if (!P0->open) P0->open = new Openings();
    Openings &O = *P0->open;
    O.reset(2 + nl);
    plan_batch(N, pos, O.plans[0]);
    O.plans[1] = O.plans[0];  // the composition tree opens the same positions
    for (int l = 0; l < nl; l++) plan_batch(l == 0 ? rows0 : layer_len[l] / fold, fri_pos[l], O.plans[2 + l]);
    // chunk requests: owner rank (-1: host top node), local buffer id, byte offset
    enum { B_LDE, B_CLDE, B_DEEP, B_TN, B_CN, B_F0N, B_FRI, B_FRI_DIG, B_TB, B_CB, B_F0B, B_CT, B_F1N, B_F1B };
    struct Req {
        int owner, buf;
        size_t off;
        const uint8_t *host;
    };
    static thread_local std::vector<Req> req;
    req.clear();
    auto lde_row = [&](int buf, int ncols, uint64_t i) {
        const int r = (int)(i & 7), own = r / Bl, j = r % Bl;
        const size_t q = i >> 3;
        for (int c = 0; c < ncols; c++) req.push_back({own, buf, 16 * (((size_t)c * Bl + j) * n + q), nullptr});
    };
    for (size_t q = 0; q < nu; q++) lde_row(B_LDE, W, pos[q]);
    for (size_t q = 0; q < nu; q++) lde_row(B_CLDE, CK, pos[q]);
    for (uint64_t rp : (nl > 0 ? fri_pos[0] : std::vector<uint64_t>())) {
        const int r = (int)(rp & 7), own = r / Bl, j = r % Bl;
        const size_t q0 = rp >> 3;
        for (uint32_t k = 0; k < fold; k++)
            for (int pln = 0; pln < KX; pln++)
                req.push_back({own, B_DEEP, 16 * ((size_t)pln * Bl * n + j * n + q0 + k * m), nullptr});
    }
    for (int l = 1; l < nl; l++) {
        const size_t L = layer_len[l], rows = L / fold;
        if (l == 1 && sh1) {  // layer 1 on the owners of its cosets: value i at CTMP [plane][j][i >> 3], coset i & 7
            for (uint64_t r : fri_pos[1])
                for (uint32_t k = 0; k < fold; k++)
                    for (int pln = 0; pln < KX; pln++) {
                        const size_t i = r + k * rows;
                        const int c = (int)(i & 7), own = c / Bl, j = c % Bl;
                        req.push_back({own, B_CT, 16 * ((size_t)pln * Bl * m + (size_t)j * m + (i >> 3)), nullptr});
                    }
            continue;
        }
        const int lb = l == lg ? lbg : 0, lcn = ilog2(L) - lb;
        for (uint64_t r : fri_pos[l])
            for (uint32_t k = 0; k < fold; k++)
                for (int pln = 0; pln < KX; pln++) {
                    const size_t i = r + k * rows, at = ((i & (((size_t)1 << lb) - 1)) << lcn) + (i >> lb);
                    req.push_back({0, B_FRI,
                                   (size_t)((const uint8_t *)(layer_vals[l] + pln * L + at) - (const uint8_t *)FRI(P0)),
                                   nullptr});
                }
    }
    const size_t off_dig = req.size();
    const DistTree *trees[4] = {&Ttrace, &Tcomp, &Tfri0, &Tfri1};
    const int tbuf[4][3] = {{-1, B_TN, B_TB}, {-1, B_CN, B_CB}, {-1, B_F0N, B_F0B}, {-1, B_F1N, B_F1B}};  // (Loc::which)
    const int ndist = sh1 ? 4 : 3;  // distributed trees: trace, composition, FRI layer 0 (and 1)
    for (int b = 0; b < 2 + nl; b++)
        for (auto &path : O.plans[b].paths)
            for (auto &e : path) {
                if (b < ndist) {
                    const DistTree::Loc L = trees[b]->locate(e.first, e.second);
                    if (L.owner < 0) {
                        const uint8_t *hp = trees[b]->top[e.second].data();
                        req.push_back({-1, 0, 0, hp});
                        req.push_back({-1, 0, 0, hp + 16});
                    } else {
                        req.push_back({L.owner, tbuf[b][L.which], L.off, nullptr});
                        req.push_back({L.owner, tbuf[b][L.which], L.off + 16, nullptr});
                    }
                } else {  // the lead's FRI layers (local rank 0 of every process, i.e. rank 0 serves)
                    const uint8_t *base = e.first ? layer_nodes[b - 2] : layer_leaves[b - 2];
                    const size_t off = (size_t)(base + 32 * e.second - P0->fri_dig);
                    req.push_back({0, B_FRI_DIG, off, nullptr});
                    req.push_back({0, B_FRI_DIG, off + 16, nullptr});
                }
            }
    const size_t NK = req.size();
    if (NK > ZK_GATHER_CAP) ZK_FAIL(ZK_ERR_INVALID_ARG, "too many opened values for the gather buffer");
    ZK_TRY(sched_entry(X, 'K', -1));  // (the lead-only segment ends: every rank gathers its openings)
    {
        std::vector<const void *> snd(nlp);
        std::vector<void *> rcv(nlp);
        for (int l = 0; l < nlp; l++) {
            zk_prover *p = X.P[l];
            const uint8_t *bases[14] = {(const uint8_t *)p->lde, (const uint8_t *)CLDE(p), (const uint8_t *)DEEP(p),
                                        p->nodes, p->cnodes, f0n[l],
                                        (const uint8_t *)FRI(p), p->fri_dig, p->sh_blk, p->sh_cblk, p->sh_fblk,
                                        (const uint8_t *)CTMP(p), f1n[l], p->sh_f1blk};
            // (the prover's pinned staging: an asynchronous copy, no wait -- the next proof on this prover writes it again
            // only after this one has drained)
            uint64_t *addr = p->h_gather_idx;
            for (size_t t = 0; t < NK; t++) {
                const Req &q = req[t];
                addr[t] = (q.owner == X.rank[l]) ? (uint64_t)(uintptr_t)(bases[q.buf] + q.off)
                                                 : (uint64_t)(uintptr_t)p->sh_zero;
            }
            ZK_CHECK_HIP(hipSetDevice(p->device));
            ZK_CHECK_HIP(hipMemcpyAsync(p->gather_idx, addr, NK * 8, hipMemcpyHostToDevice, p->st));
            gather_chunks(p->st, p->gather_idx, NK, p->gather_out);
            snd[l] = p->gather_out;
            rcv[l] = p->sh_buf;
        }
        ZK_TRY(xchg(X, "openings", AG, snd, rcv, NK * sizeof(fe)));
    }
    std::vector<fe> all((size_t)G * NK), got(NK);
    ZK_CHECK_HIP(hipMemcpyAsync(all.data(), P0->sh_buf, all.size() * sizeof(fe), hipMemcpyDeviceToHost, P0->st));
    ZK_CHECK_HIP(hipStreamSynchronize(P0->st));
    for (size_t t = 0; t < NK; t++) {
        if (req[t].owner < 0)
            memcpy(&got[t], req[t].host, 16);
        else
            got[t] = all[(size_t)req[t].owner * NK + t];
    }
    {
        size_t off = 0;
        O.trace_rows.assign(got.begin(), got.begin() + nu * W);
        off += nu * W;
        O.comp_rows.assign(got.begin() + off, got.begin() + off + nu * CK);
        off += nu * CK;
        for (int l = 0; l < nl; l++) {
            O.fri_rows[l].assign(got.begin() + off, got.begin() + off + fri_pos[l].size() * fold * KX);
            off += fri_pos[l].size() * fold * KX;
        }
        const uint8_t *dg = (const uint8_t *)(got.data() + off_dig);
        for (int b = 0; b < 2 + nl; b++) {
            const size_t bytes = 32 * O.plans[b].count();
            O.digests[b].assign(dg, dg + bytes);
            dg += bytes;
        }
    }
    stage_mark(P0, "queries");
    const std::vector<uint8_t> bytes = serialize_proof(n, opt, C, R, h.data(), O, KX == 2 ? &rem_flat : nullptr);
    stage_mark(P0, "serialize");
    ZK_CHECK_HIP(hipStreamSynchronize(P0->st));
    stage_collect(P0);
    collect_kernel_stats(P0);
    if (rec) *rec = R;
    return deliver_proof(bytes, degree_flag, proof_out, proof_len);
}

}  // namespace

// ---------------------------------------------------------------- C ABI
int zk_comm_create_loopback(int world, zk_comm **out) {
    if (!out || (world != 1 && world != 2 && world != 4 && world != 8))
        ZK_FAIL(ZK_ERR_INVALID_ARG, "world must be 1, 2, 4 or 8 (ranks own 8/world cosets)");
    auto *c = new LoopbackComm();
    c->world = world;
    c->rank = 0;
    *out = c;
    return ZK_OK;
}

int zk_comm_unique_id(uint8_t id[128]) {
    if (!id) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    return zk_rccl_unique_id(id);
}

int zk_comm_create_rccl(const uint8_t id[128], int rank, int world, int device, zk_comm **out) {
    if (!id || !out || rank < 0 || rank >= world || (world != 1 && world != 2 && world != 4 && world != 8))
        ZK_FAIL(ZK_ERR_INVALID_ARG, "invalid rank / world (world must be 1, 2, 4 or 8)");
    return zk_make_rccl_comm(id, rank, world, device, out);
}

int zk_comm_create_host(int rank, int world, zk_exchange_fn fn, void *ctx, zk_comm **out) {
    if (!fn || !out || rank < 0 || rank >= world || (world != 1 && world != 2 && world != 4 && world != 8))
        ZK_FAIL(ZK_ERR_INVALID_ARG, "invalid rank / world (world must be 1, 2, 4 or 8) or null callback");
    auto *c = new HostComm();
    c->world = world;
    c->rank = rank;
    c->fn = fn;
    c->ctx = ctx;
    *out = c;
    return ZK_OK;
}

void zk_comm_destroy(zk_comm *c) { delete c; }

int zk_comm_set_trace_split(zk_comm *c, int replicated) {
    if (!c) ZK_FAIL(ZK_ERR_INVALID_ARG, "null communicator");
    if (replicated < -1) ZK_FAIL(ZK_ERR_INVALID_ARG, "replicated columns: -1 (default) or a count");
    c->split_rep = replicated;
    return ZK_OK;
}

int zk_comm_set_measure(zk_comm *c, int on) {
    if (!c) ZK_FAIL(ZK_ERR_INVALID_ARG, "null communicator");
    if (!c->loopback()) ZK_FAIL(ZK_ERR_INVALID_ARG, "the measurement mode needs a loopback communicator");
    c->measure = on != 0;
    return ZK_OK;
}

int zk_prove_sharded(zk_comm *comm, zk_prover **provers, int nlocal, const uint8_t *trace, size_t n,
                     const zk_options *opt, const zk_pub_inputs *pub, uint8_t *proof_out, size_t *proof_len,
                     zk_record *rec) {
    return zk::prove_sharded_entry(comm, provers, nlocal, trace, n, opt, pub, proof_out, proof_len, rec, nullptr);
}

int zk::shard_rank_of(const zk_comm *comm, int l) { return comm->loopback() ? l : comm->rank; }

int zk::prove_sharded_entry(zk_comm *comm, zk_prover **provers, int nlocal, const uint8_t *trace, size_t n,
                            const zk_options *opt, const zk_pub_inputs *pub, uint8_t *proof_out, size_t *proof_len,
                            zk_record *rec, const FixedCols *fixed) {
    if (!comm || !provers || !proof_len || nlocal <= 0) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    if (fixed && trace) ZK_FAIL(ZK_ERR_INVALID_ARG, "preprocessed columns go with a device trace");
    if (comm->loopback() ? nlocal != comm->world : nlocal != 1)
        ZK_FAIL(ZK_ERR_INVALID_ARG,
                "a loopback communicator needs one prover per rank, an RCCL or host-exchange one exactly one");
    Ctx X;
    X.comm = comm;
    X.G = comm->world;
    X.Bl = 8 / X.G;
    X.n = n;
    for (int l = 0; l < nlocal; l++) {
        zk_prover *p = provers[l];
        if (!p) ZK_FAIL(ZK_ERR_INVALID_ARG, "null prover");
        if (p->shard_world && p->shard_world != X.G)
            ZK_FAIL(ZK_ERR_INVALID_ARG, "prover was created for a sharded proof over a different number of ranks");
        ZK_TRY(check_prove_args(n, p->max_n, p->max_b, opt, pub));
        X.P.push_back(p);
        X.rank.push_back(comm->loopback() ? l : comm->rank);
    }
    if (opt->blowup != 8) ZK_FAIL(ZK_ERR_INVALID_ARG, "the sharded prover needs blowup 8 (LDE cosets = CE cosets)");
    const size_t m = n / opt->fri_folding;
    if (m < 8 * (size_t)X.G || n / X.G < 8) ZK_FAIL(ZK_ERR_INVALID_ARG, "trace too short to shard over this many ranks");
    X.log_n = ilog2(n);
    X.C = num_comp_cols(n);
    if (X.C > 8) ZK_FAIL(ZK_ERR_INVALID_ARG, "composition column count exceeds 8");
    for (auto *p : X.P) {
        ZK_CHECK_HIP(hipSetDevice(p->device));
        Plan *pl = nullptr;
        ZK_TRY(get_plan(p, n, 8, &pl));
        ZK_TRY(plan_rank_tables(p, pl, X.rank[X.pl.size()] * X.Bl, X.G));  // its fill tables over this rank's cosets
        X.pl.push_back(pl);
        if (opt->field_extension == 2) ZK_TRY(ensure_ext(p));
        if (!p->sh_buf) {
            ZK_CHECK_HIP(p->arena.alloc(&p->sh_buf, (size_t)8 * ZK_GATHER_CAP));
            ZK_CHECK_HIP(p->arena.alloc(&p->sh_xr, 8));
            ZK_CHECK_HIP(p->arena.alloc(&p->sh_zero, 1));
            ZK_CHECK_HIP(p->arena.alloc(&p->sh_roots, 32 * 8));
            ZK_CHECK_HIP(p->arena.alloc(&p->sh_flags, 8));
            ZK_CHECK_HIP(hipMemset(p->sh_zero, 0, sizeof(fe)));
            // a rank-sized prover's Bl cosets; a full prover may serve any G >= 2 (Bl <= 4)
            const size_t bl = p->shard_world ? (size_t)8 / p->shard_world : 4, mn = p->max_n;
            ZK_CHECK_HIP(p->arena.alloc(&p->sh_blk, 32 * (2 * bl - 1) * mn));
            ZK_CHECK_HIP(p->arena.alloc(&p->sh_cblk, 32 * (2 * bl - 1) * mn));
            ZK_CHECK_HIP(p->arena.alloc(&p->sh_fblk, 32 * (2 * bl - 1) * (mn / 2)));
            ZK_CHECK_HIP(p->arena.alloc(&p->sh_f1blk, 32 * (2 * bl - 1) * (mn / 4)));
        }
    }
    // one rank: nothing to shard or exchange, so the single-GPU path proves it (the same proof bytes; its
    // seven-coset evaluation only pays off without ranks to balance: DESIGN.md section 7, round 4)
    if (X.G == 1)
        return fixed ? prove_fixed(X.P[0], n, opt, pub, fixed, proof_out, proof_len)
                     : prove_single(X.P[0], trace, n, opt, pub, proof_out, proof_len, rec);
    X.fixed = fixed;
    // measurement mode (loopback): every rank's kernels on rank 0's stream, in program order (restored on the way out)
    struct SharedStream {
        std::vector<zk_prover *> P;
        std::vector<hipStream_t> own;
        ~SharedStream() {
            for (size_t l = 1; l < P.size(); l++) {
                (void)hipStreamSynchronize(P[l]->st);
                P[l]->st = own[l];
            }
        }
    } shared;
    if (comm->measure) {
        for (auto *p : X.P) {
            // (work the caller queued on a rank's own stream -- zk_vm_prove_sharded's trace rows -- completes first)
            ZK_CHECK_HIP(hipSetDevice(p->device));
            ZK_CHECK_HIP(hipStreamSynchronize(p->st));
            shared.P.push_back(p);
            shared.own.push_back(p->st);
        }
        for (size_t l = 1; l < X.P.size(); l++) X.P[l]->st = X.P[0]->st;
    }
    X.P[0]->sched_world = X.G;
    X.P[0]->sched_measure = comm->measure;
    // every local rank's proof counts as in flight on its device (the single-GPU AUTO upload schedule reads it)
    std::vector<std::unique_ptr<DeviceBusy>> busy;
    for (auto *p : X.P) busy.push_back(std::make_unique<DeviceBusy>(p->dev_busy));
    // drop any staged reads an earlier failed proof left behind, and again on every way out of this one
    std::vector<std::unique_ptr<IoScope>> io_scopes;
    for (auto *p : X.P) {
        ZK_CHECK_HIP(hipSetDevice(p->device));
        io_scopes.push_back(std::make_unique<IoScope>(p));
    }
    const size_t cap = *proof_len;  // (in/out)
    int rc = prove_sharded(X, trace, opt, pub, proof_out, proof_len, rec);
    if (rc == ZK_SH_REDO) {
        *proof_len = cap;
        // a hinted column was not what the previous proof found (every rank saw the same all-gathered checks): forget
        // the hints (and stop speculating the clock at this length if it was refuted), prove from every column
        for (zk_prover *p : X.P) {
            p->sh_hint_n = 0;
            p->sh_sparse = p->sh_nw8 = p->sh_nw32 = 0;
            p->sh_clock = false;
            if (X.sh_clock && (X.sh_refuted & 1u)) p->sh_clock_off_n = n;
        }
        X.hint_ok = false;
        X.sh_refuted = 0;
        rc = prove_sharded(X, trace, opt, pub, proof_out, proof_len, rec);
    }
    return rc;
}
