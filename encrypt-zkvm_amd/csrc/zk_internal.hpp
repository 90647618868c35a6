// zk_internal.hpp -- shared declarations of the gfx950 prove path (kernels.hip, prover.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "ext2.hpp"
#include "f128.hpp"

namespace zk {

// ---------------------------------------------------------------- kernel profiler
// When enabled, every kernel launch is bracketed by a pair of HIP events on its own stream, so
// per-kernel device time is measured on the stream the kernel actually runs on.
struct KernelProfiler {
    bool on = false;
    struct Rec {
        const char *name;
        hipEvent_t a, b;
        double bytes;  // algorithmic HBM bytes of this launch (DESIGN.md "Roofline accounting")
        double muls, addsubs;  // algorithmic f128 multiplies / additions+subtractions (0 = not modelled)
    };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    hipEvent_t get() {
        if (used == pool.size()) {
            hipEvent_t e;
            hipEventCreate(&e);
            pool.push_back(e);
        }
        return pool[used++];
    }
    void begin(hipStream_t st, const char *name, double bytes, double muls = 0, double addsubs = 0) {
        Rec r{name, get(), nullptr, bytes, muls, addsubs};
        hipEventRecord(r.a, st);
        recs.push_back(r);
    }
    void end(hipStream_t st) {
        recs.back().b = get();
        hipEventRecord(recs.back().b, st);
    }
    void reset() {
        recs.clear();
        used = 0;
    }
};
KernelProfiler &profiler();
// ZK_PROF with the launch's algorithmic f128 operation counts (for the VALU roofline)
#define ZK_PROF_OPS(st, name, bytes, muls, addsubs, ...)                               \
    do {                                                                             \
        ::zk::KernelProfiler &P_ = ::zk::profiler();                                 \
        if (P_.on) P_.begin(st, name, (double)(bytes), (double)(muls), (double)(addsubs)); \
        __VA_ARGS__;                                                                 \
        if (P_.on) P_.end(st);                                                       \
    } while (0)
#define ZK_PROF(st, name, bytes, ...)        \
    do {                                     \
        ::zk::KernelProfiler &P_ = ::zk::profiler(); \
        if (P_.on) P_.begin(st, name, (double)(bytes)); \
        __VA_ARGS__;                         \
        if (P_.on) P_.end(st);               \
    } while (0)

// ---------------------------------------------------------------- twiddle plans
// Every power table the kernels need for one NTT size n, resident in HBM.
//   dft_fwd / dft_inv : w_4096^t, t < 2048  (DFT stages of the in-LDS engine; smaller sizes stride)
//   big_lo / big_hi   : w_n^t = big_lo[t & 2047] * big_hi[t >> 11]  (inter-pass twiddles, x values)
struct NttTables {
    int log_n = 0;
    fe *dft_fwd = nullptr, *dft_inv = nullptr;
    fe_ws *dft_fwd_ws = nullptr, *dft_inv_ws = nullptr;  // their W sets (f128.hpp fe_mul_uniform)
    fe_w2 *dft_fwd_w2 = nullptr, *dft_inv_w2 = nullptr;  // and two-part forms (f128.hpp fe_mul_w2)
    fe *fwd_lo = nullptr, *fwd_hi = nullptr, *inv_lo = nullptr, *inv_hi = nullptr;
    // four-step inter-pass twiddles w^(j2*k1) laid out as pass 1 consumes them, [k1 * n2 + j2]
    // (n elements each; only for log_n > 12, else null)
    fe *fwd_pass = nullptr, *inv_pass = nullptr;
    // optional: inv_pass * n^-1, used when an inverse NTT is post-scaled by n^-1 (interpolation): the
    // scale rides on the pass-1 twiddle instead of costing a multiply per element in pass 2
    fe *inv_pass_n = nullptr;
    fe inv_n = {0, 0};
};
// Four-step split of a size-2^L NTT (L > 12): log2 of the pass-1 line length n2 (pass-2 lines are
// n1 = 2^(L - log_n2)).  Pass 1 reads strided and writes contiguous runs; pass 2 reads and writes
// LPB-element row segments at stride n2, so pass 2 gets the shorter lines when the split is uneven:
// at L = 22 the balanced 11/11 split leaves pass 2 with 32-B segments (2 lines of 2048 per
// 4096-element tile) and an extra radix-2 LDS stage; 12/10 gives it the 64-B segments of 2^20.
// Every table builder and the NTT dispatcher use this one function, so they always agree.
// (the balanced ceil(L/2) split measured slower at 2^22: DESIGN.md "NTT")
int ntt_log_n2(int L);
// fill NttTables::fwd_pass / inv_pass (allocated by the caller, n elements each)
void make_pass_twiddles(hipStream_t st, NttTables &T);
// out[k1*n2 + j2] = s^k1 * fwd_pass[k1*n2 + j2] (s^t from split tables): CosetTables::pass of one coset
void coset_pass_tables(hipStream_t st, const fe *s_lo, const fe *s_hi, const fe *fwd_pass, int log_n, int log_n2,
                       fe *out);

// A power series s^k, k < n, as split tables (s^k = lo[k & 2047] * hi[k >> 11])
struct PowTable {
    fe *lo = nullptr, *hi = nullptr;  // s^t = lo[t & 2047] * hi[t >> 11]
    fe *full = nullptr;               // optional s^t for every t < n (one multiply less per use)
};
// out[t] = lo[t & 2047] * hi[t >> 11] for t < n
void pow_expand(hipStream_t st, const fe *lo, const fe *hi, size_t n, fe *out);

// Sparse columns of a trace batch: column c (flags at nz[col0 + c]) is zero in every row but the last when
// nz[col0 + c] == 0 (sparse_detect); then its interpolation is last[col0 + c] * lagr (the interpolant of e_(n-1))
// and its coset LDE last * lagr_lde (coset r at r n): the NTT passes skip its DFTs.  Four-step sizes only.
struct SparseCols {
    const unsigned *nz;
    const fe *last;
    const fe *lagr, *lagr_lde;
    int col0;
    // width flags (sparse_detect only): wstride > 0 sets nz[wstride + c] when column c has an entry of 8 bits or more
    // and nz[2 wstride + c] when one of 32 bits or more (last row excluded) -- the next proof's narrow-upload hint
    int wstride = 0;
    // fused: the interpolation's pass 1 writes the flags (nz, and with wstride the width flags) of the columns it
    // reads and skips none; the coset LDE then skips none either (host-resident traces once the hints are learned:
    // no separate detection pass over the uploaded columns)
    bool fused = false;
    // all: the host knows every column of the call is sparse (the hinted columns of a host trace): no transform is
    // launched, one streaming pass writes last * fill into every column (k_sparse_fill)
    bool all = false;
    // idoff > 0: column 0 is also checked for being the AIR clock (rows 0 .. n-2 hold 0 .. n-2; nz[idoff] = 1 when it
    // is not); such a column transforms to id + (last - (n-1)) * fill (id_poly / id_lde: the identity column's
    // interpolant and coset LDE, like lagr / lagr_lde) and skips its DFTs like a sparse one
    const fe *id_poly = nullptr, *id_lde = nullptr;
    int idoff = 0;
    // the cosets lagr_lde / id_lde hold: coset r at slot (r - lde_r0) >> lde_shift (Plan::lde_slot)
    int lde_r0 = 0, lde_shift = 0;
};
void sparse_detect(hipStream_t st, const fe *trace, size_t n, int c0, int nc, const SparseCols &sp);
void sparse_detect_rows(hipStream_t st, const fe *trace, size_t n, int c0, int nc, const SparseCols &sp, size_t r0,
                        size_t r1);
// Narrow trace columns uploaded packed (zk_prove from host columns): column col[k]'s rows 0 .. n-2 as width[k]-byte
// integers (1 or 4) at src + off[k], its last row last[k]; written out as field elements into trace column col[k].
struct NarrowCols {
    int count;
    int col[28];
    int width[28];
    size_t off[28];
    fe last[28];
};
void expand_narrow(hipStream_t st, const uint8_t *src, const NarrowCols &nc, size_t n, fe *trace);

// NTT of `batch` polynomials of size 2^log_n, each at in + b*in_stride -> out + b*out_stride.
//   inverse     : use w^-1 (no 1/n scale; fold it into post_scale)
//   pre         : optional s^k pre-scale of input coefficient k (coset evaluation), may be null
//   post_scale  : optional constant multiplied into every output (e.g. 1/n)
// in and out must not alias.  tmp must hold batch * n elements when log_n > 12.
// sp (optional, interpolations with post_scale = 1/n only): sparse columns of the batch (SparseCols)
void ntt(hipStream_t st, const NttTables &T, const fe *in, size_t in_stride, fe *out, size_t out_stride,
         int batch, bool inverse, const PowTable *pre, const fe *post_scale, fe *tmp, const SparseCols *sp = nullptr);

// Coset-LDE tables of one plan (LDE coset r < B, s_r = 3 w_N^r):
//   n <= 4096 (single pass): full[r*n + k] = s_r^k (input pre-scale)
//   four-step (n = n1*n2):   stage[r*4096 + h + j] = c_r^(n2/2h) w_2h^j, c_r = s_r^n1 (DIT stage twiddles of
//                            the pass-1 line DFT over the coset c_r <w_n2>), pass[r*n + k1*n2 + j2] = (s_r w_n^j2)^k1
struct CosetTables {
    fe *full = nullptr, *stage = nullptr, *pass = nullptr;
    fe_ws *stage_ws = nullptr;  // W sets of `stage` (four-step plans)
    fe_w2 *stage_w2 = nullptr;  // two-part forms of `stage`
};
// Forward coset LDE: for columns c < ncols (at in + c*in_stride) and coset slots j < ncos (coset r0 + j*rstride),
// the n evaluations over coset r to out + c*out_cstride + j*out_jstride.  tmp: ncols*min(ncos, 8)*n
// (four-step; launches of up to 8 cosets).
void ntt_lde(hipStream_t st, const NttTables &T, const CosetTables &CT, const fe *in, size_t in_stride, int ncols,
             int r0, int rstride, int ncos, fe *out, size_t out_cstride, size_t out_jstride, fe *tmp,
             const SparseCols *sp = nullptr);
// out[i] = F[i] + d * L[i] for i < cnt (d given by its W set)
void axpy_fill(hipStream_t st, const fe *F, const fe *L, const fe_ws &d, size_t cnt, fe *out);

// grinding: atomicMin into *best_dev of the nonces in [start, start+count) with >= bits trailing zeros
void grind_launch(hipStream_t st, const uint32_t *seed_dev, uint64_t start, uint32_t count, int bits,
                  unsigned long long *best_dev);

// ---------------------------------------------------------------- hashing
// leaf[i] = BLAKE3(row i) for natural LDE index i < N = B*n of a coset-major column set:
// element (column c, index i) lives at base[(c*B + i%B)*n + i/B].
// leaves (N x 32 B) and the heap-ordered Merkle tree nodes[1..N) of coset-major rows / FRI layer rows
// leaf digests of the rows of LDE cosets r0 .. r0 + 2^log_rc - 1 (coset-major columns), natural leaf order
void hash_rows_cosets(hipStream_t st, const fe *base, int ncols, int log_n, int log_b, int r0, int log_rc,
                      uint8_t *leaves);
void commit_rows_coset_major(hipStream_t st, const fe *base, int ncols, int log_n, int log_b, uint8_t *leaves,
                             uint8_t *nodes);
// blocks b0 .. b1 - 1 of the leaf hashes of all B n rows of a coset-major column set of ncols (a multiple of 4,
// <= 64) columns: columns 4 b .. 4 b + 3 compressed into the chaining value each leaf slot carries between launches
// Virtual trace columns (host traces, prover.hip): sparse columns whose LDE is never written; the row hashing forms
// column c's value at LDE point (coset r, position q) as last[c] * lagr_lde[r n + q]
struct VirtCols {
    uint32_t mask = 0;
    const fe *last = nullptr, *lagr_lde = nullptr;
};
void hash_rows_blocks(hipStream_t st, const fe *base, int ncols, int log_n, int log_b, int b0, int b1, uint8_t *leaves,
                      VirtCols virt = VirtCols());
// Storage of a FRI layer of L values: natural order (lb = 0), or coset-major over 2^lb cosets of 2^lcn
// points (natural index i at (i mod 2^lb) 2^lcn + i / 2^lb): layer 0 as the DEEP coset LDE leaves it
struct FriLayout {
    int lb, lcn;
};
FriLayout fri_layout(size_t L, int lb);
// FRI layer leaves: row r of a layer of size L (rows = L/fold): [e[r + k*L/fold]]
void commit_fri_layer(hipStream_t st, const fe *layer, size_t L, int fold, uint8_t *leaves, uint8_t *nodes, int lb = 0);
// nodes[1..nl) of a binary Merkle tree over nl leaves (nodes[nl/2..nl) = merges of leaf pairs)
void merkle_tree(hipStream_t st, const uint8_t *leaves, size_t nl, uint8_t *nodes);
// out[k] = src[idx[k]] for 32-byte digests
// out[t] = the 16 bytes at device address addr[t] (query openings: LDE values and Merkle digests)
constexpr size_t ZK_GATHER_CAP = 1 << 17;
void gather_chunks(hipStream_t st, const uint64_t *addr, size_t k, fe *out);
// Up to ZK_COPY_LIST_MAX device -> pinned-host copies (32-bit words) in one launch: blockIdx.y picks
// the entry.  dst must be host memory from hipHostMalloc (device-accessible, coherent).
constexpr int ZK_COPY_LIST_MAX = 32;
struct CopyList {
    int n;
    const uint32_t *src[ZK_COPY_LIST_MAX];
    uint32_t *dst[ZK_COPY_LIST_MAX];
    uint32_t words[ZK_COPY_LIST_MAX];
};
hipError_t copy_to_host(hipStream_t st, const CopyList &L, size_t max_words);
void gather_digests(hipStream_t st, const uint8_t *src, const uint64_t *idx, size_t k, uint8_t *out);
// out[q*ncols + c] = element (c, pos[q]) of a coset-major column set
void gather_rows(hipStream_t st, const fe *base, int ncols, int log_n, int log_b, const uint64_t *pos, size_t k,
                 fe *out);

// ---------------------------------------------------------------- AIR / composition
struct AirConsts {
    fe coeff_t[20];
    fe coeff_b[22];
    int assert_col[22];
    int assert_grp[22];  // 0: step 0, 1: step n-2
    fe assert_val[22];
    fe inv_zn[8];   // 1 / (x^n - 1) on the 8 CE cosets
    fe xr[8];       // 3 * w_CE^r
    fe g_last2, g_last1;
    fe delta;
    fe bnd1;  // sum_k coeff_b[12+k] * assert_val[12+k]: the step n-2 group's values, subtracted once per row
    int lwe_size;
};
// inverse of (x - a) * (x - b) over the B cosets, written coset-major: out[r*n + q] for the point
// x = xr[r] * w_n^q (natural domain index i = r + B*q)
void batch_inv_pairs(hipStream_t st, const NttTables &Tn, const fe *xr, int log_b, int log_n, fe a, fe b,
                     fe *out);
struct Fe8 {
    fe v[8];
};
// The evaluator's per-row divisor factors over 2^log_cos cosets (offsets xr, coset-major, planes of
// P = 2^(log_cos + log_n)): out[i] = (x - g2)(x - g1) inv_zn[coset], out[P + i] = 1/(x - 1),
// out[2P + i] = 1/(x - g2); inv_zn[c] = 1/(xr[c]^n - 1).  3P elements.
void divisor_tables(hipStream_t st, const NttTables &Tn, const fe *xr, int log_cos, int log_n, fe g1, fe g2,
                    const Fe8 &inv_zn, fe *out);
// Which CE cosets one launch evaluates: local coset jl < nce is global CE coset ce0 + cestep*jl, and its
// LDE rows are LDE coset slot jl << lshift of a buffer holding lde_cosets cosets per column.  dplane: the stride of
// the divisor tables' planes (0: nce * n, the launch's own cosets; a launch over one coset of several passes theirs).
struct EvalMap {
    int nce, ce0, cestep, lshift, lde_cosets;
    size_t dplane = 0;
};
// Rescue MDS / inverse-MDS __constant__ tables on the current device (once per device; thread-safe).
// zk_prover_create calls it; the evaluator launches check it again (the plug point may run first).
hipError_t upload_rescue_consts(hipStream_t st);
// bnd: the boundary (assertion) terms are evaluated per row (else: boundary_poly_add after interpolation)
hipError_t eval_constraints_mapped(hipStream_t st, const fe *lde, int log_n, EvalMap map, const fe *periodic,
                             const fe *divs, const AirConsts *consts_dev, fe *comp, bool bnd = true);
// Inputs of the cross-coset step for coefficients k0 .. k0+kcount: c[r][kl] = c_r[k0 + kl]; output
// polys[k2 * pstride + kl].
struct CrossMap {
    const fe *c[8];
    size_t k0, kcount, pstride;
    // derive7: coset 7 was not evaluated (c[7] unused).  A composition polynomial of degree < 7n has a zero
    // top block, b_7 = sum_r w8^(7r) ... = 0, which fixes d_7 = sum_{r<7} k7[r] d_r with k7[r] = -w_8^(r+1).
    int derive7 = 0;
    fe k7[7] = {};
};
void comp_cross_mapped(hipStream_t st, const CrossMap &m, const NttTables &T8n, const PowTable &inv3, fe scale,
                       fe w8inv, fe inv3n, int ncols, fe *polys, unsigned *nonzero_flag);
// composition evaluations over the CE domain (8n), written coset-major: comp[r*n + q], i = 8q + r
// nce: evaluate CE cosets 0 .. nce-1 (8: all; 7: the composition stage derives the last one, bnd = false)
hipError_t eval_constraints(hipStream_t st, const fe *lde, int log_n, int log_b, const fe *periodic, const fe *divs,
                      const AirConsts *consts_dev, fe *comp, bool bnd = true, int nce = 8);
// add the boundary terms' quotient polynomial (one coefficient plane K) into col0 (n coefficients);
// c = g^(n-2); scratch: deep_poly's layout; sets *flag when an assertion fails
void boundary_poly_add(hipStream_t st, const fe *tpolys, int log_n, const AirConsts &K, fe c, fe *scratch, fe *col0,
                       unsigned *flag);
// boundary_poly_add split over a sharded rank's coefficient range [k0, k0 + kn) (kn a multiple of
// ZK_DEEP_RANGE_QUANTUM): begin -> the range's 2 sums on the device; end adds the quotient's range into col0
// (global index) given ext = the sums of every later range.  The remainder flag is raised by the rank with k0 = 0.
const fe *boundary_range_begin(hipStream_t st, const fe *tpolys, int log_n, const AirConsts &K, fe c, fe *scratch,
                               size_t k0, size_t kn);
void boundary_range_end(hipStream_t st, int log_n, fe c, fe *scratch, size_t k0, size_t kn, const fe *ext, fe *col0,
                        unsigned *flag);
// cross-coset step of the size-8n interpolation: per k1 < n, from the 8 per-coset inverse NTTs
// (c_r[k1]), produce coefficients a[k1 + n*k2] = 3^-(k1+n k2) / (8n) * sum_r w8^(-r k2) w_8n^(-r k1) c_r[k1]
// and write column k2 < ncols of the segmented composition polynomial: polys[k2*n + k1].
void comp_cross_coset(hipStream_t st, const fe *c, int log_n, const NttTables &T8n, const PowTable &inv3,
                      fe scale, fe w8inv, fe inv3n, int ncols, fe *polys, unsigned *nonzero_flag);

// ---------------------------------------------------------------- OOD / DEEP / FRI
// out[p*2 + 0/1 ...]: evaluate `npolys` polys (n coeffs, stride n) at point x; partial sums per block
// OOD frame in one pass: out = [T_c(z)]_W ++ [T_c(zg)]_W ++ [H_j(z)]_C.  tab: 128 + 2*ood_waves(n)
// elements, partials: (2W + C) * ood_waves(n) elements of scratch.
int ood_waves(size_t n);
void ood_eval(hipStream_t st, const fe *tpolys, int W, const fe *cpolys, int C, int log_n, fe z, fe zg, fe *tab,
              fe *partials, fe *out, int rank = 0, int G = 1);
void sum_partials(hipStream_t st, const fe *partials, int npolys, int nblk, fe *out, int b0 = 0, int b1 = -1);
// DEEP over the LDE domain, natural order (consts: DeepConsts in device memory)
struct DeepConsts {
    fe alpha_t[32];
    fe alpha_c[16];
    fe k1, k2, z, zg;
};
// LDE of one n-coefficient polynomial over `count` cosets r0 + stride*j: out[j*n ..], coset-major.  ntt_tmp: 8n.
void lde_cosets(hipStream_t st, const NttTables &Tn, const CosetTables &CT, const fe *coeffs, size_t n, size_t r0,
                size_t stride, int count, fe *out, fe *ntt_tmp);
// The DEEP polynomial's coefficients (n; over E two planes of n) computed into scratch (returned)
const fe *deep_poly(hipStream_t st, const fe *tpolys, const fe *cpolys, int ccols, int log_n,
                    const void *deep_consts_dev, fe z, fe zg, fe *scratch);
const fe *deep_poly_ext(hipStream_t st, const fe *tpolys, const fe *cpolys, int ccols, int log_n,
                        const void *deep_consts_dev, fe2 z, fe2 zg, fe *scratch);
// The same split by coefficient range over the ranks of a sharded proof: rank g computes the range [k0, k0 + kn)
// (kn a multiple of ZK_DEEP_RANGE_QUANTUM) in two steps around one exchange.  deep_range_begin returns a device
// pointer to the range's totals (2 base elements; over E 4); deep_range_end takes `ext`, the sum of the totals of
// every later range (the suffix carried into this one), and returns the coefficient buffer (n; over E two planes of
// n) with this range filled in.  The scratch is deep_poly's.
constexpr size_t ZK_DEEP_RANGE_QUANTUM = 2048;
const fe *deep_range_begin(hipStream_t st, const fe *tpolys, const fe *cpolys, int ccols, int log_n,
                           const void *deep_consts_dev, fe z, fe zg, fe *scratch, size_t k0, size_t kn);
const fe *deep_range_end(hipStream_t st, int log_n, fe z, fe zg, fe *scratch, size_t k0, size_t kn, const fe *ext);
const fe *deep_range_begin_ext(hipStream_t st, const fe *tpolys, const fe *cpolys, int ccols, int log_n,
                               const void *deep_consts_dev, fe2 z, fe2 zg, fe *scratch, size_t k0, size_t kn);
const fe *deep_range_end_ext(hipStream_t st, int log_n, fe2 z, fe2 zg, fe *scratch, size_t k0, size_t kn,
                             const fe *ext);
// DEEP through coefficient form (kernels.hip): the DEEP polynomial (S - S(z))/(x - z) + (A - A(zg))/(x - zg)
// by suffix sums over the combined coefficients, one LDE over the B cosets (CosetTables) into ulde
// (coset-major), and (out != nullptr) a natural-order copy in out.  scratch: 4 (2048 + n/2048 + 2) + 3n + 2 ceil(n/256)
// elements; ulde: B*n; ntt_tmp: 8n.
void deep_coeff_launch(hipStream_t st, const NttTables &Tn, const fe *tpolys, const fe *cpolys, int ccols, int log_n,
                       int log_b, const void *deep_consts_dev, fe z, fe zg, const CosetTables &CT, fe *scratch,
                       fe *ulde, fe *ntt_tmp, fe *out);
// the same over E (FieldExtension::Quadratic; DeepConstsE): scratch 8 (2048 + n/2048 + 2) + 6n + 4 ceil(n/256)
// elements; ulde: 2*B*n; out planar (2N)
void deep_coeff_ext_launch(hipStream_t st, const NttTables &Tn, const fe *tpolys, const fe *cpolys, int ccols,
                           int log_n, int log_b, const void *deep_consts_dev, fe2 z, fe2 zg, const CosetTables &CT,
                           fe *scratch, fe *ulde, fe *ntt_tmp, fe *out);
// FRI fold: next[r] = p_r(alpha) over rows r < L/fold (consts: FoldConsts in device memory)
struct FoldConsts {
    fe zinv[16];  // zeta^-t, t < fold
    fe alpha, inv_offset, inv_fold;
};
void fri_fold_launch(hipStream_t st, const fe *layer, size_t L, int fold, const void *fold_consts_dev,
                     const NttTables &TN, size_t wstride, fe *next, int lb = 0);
void coset_major_to_natural(hipStream_t st, const fe *src, int log_n, int log_b, fe *dst);
// FRI commit-phase coin on the device: seed = merge(seed, root_dev), alpha (k = 1 or 2 components) drawn
// into alpha_dev (where the fold reads it) and alpha_log (the per-layer record the host replay is checked
// against)
void fri_coin_launch(hipStream_t st, uint32_t *seed_dev, const uint8_t *root_dev, int k, fe *alpha_dev,
                     fe *alpha_log);

// ---------------------------------------------------------------- FieldExtension::Quadratic (ext2.hpp)
// Every E-valued buffer is planar: component a at [0, M), component b at [M, 2M).
// OOD frame over E points: out[j*np + P], np = 2W + C, component j of poly P's value (T(z), T(zg), H(z));
// tab: 2 * (128 + 2 * ood_waves(n)) fe, partials: 2 * np * ood_waves(n) fe.
void ood_eval_ext(hipStream_t st, const fe *tpolys, int W, const fe *cpolys, int C, int log_n, fe2 z, fe2 zg,
                  fe *tab, fe *partials, fe *out, int rank = 0, int G = 1);
// composition over E: consts2_dev = {a components, b components}; planes comp[0, 8n), comp[8n, 16n)
hipError_t eval_constraints_ext(hipStream_t st, const fe *lde, int log_n, int log_b, const fe *periodic, const fe *divs,
                          const AirConsts *consts2_dev, fe *comp, bool bnd = true, int nce = 8);
// ... over the CE cosets of `map` (see eval_constraints_mapped), b plane at comp + plane
hipError_t eval_constraints_ext_mapped(hipStream_t st, const fe *lde, int log_n, EvalMap map, const fe *periodic,
                                 const fe *divs, const AirConsts *consts2_dev, size_t plane, fe *comp, bool bnd = true);
// out[i] = 1 / (N(x_i - z) N(x_i - zg)), N the norm E -> F (coset-major like batch_inv_pairs)
void batch_inv_norm_pairs(hipStream_t st, const NttTables &Tn, const fe *xr, int log_b, int log_n, fe2 z, fe2 zg,
                          fe *out);
struct DeepConstsE {
    fe2 alpha_t[32];
    fe2 alpha_c[16];
    fe2 k1, k2, z, zg;
    fe zb2, zgb2;  // z.b^2, zg.b^2
};
struct FoldConstsE {
    fe zinv[16];
    fe2 alpha;
    fe inv_offset, inv_fold;
};
// layer planar (2L), next planar (2 L/fold); leaves hash rows of fold E values (a, b per value)
void commit_fri_layer_ext(hipStream_t st, const fe *layer, size_t L, int fold, uint8_t *leaves, uint8_t *nodes, int lb = 0);
void fri_fold_ext_launch(hipStream_t st, const fe *layer, size_t L, int fold, const void *fold_consts_dev,
                         const NttTables &TN, size_t wstride, fe *next, int lb = 0);
// out[k] = src[idx[k]] for field elements
void gather_fe(hipStream_t st, const fe *src, const uint64_t *idx, size_t k, fe *out);

}  // namespace zk

namespace zk {
void diag_field_op(hipStream_t st, int op, const fe *a, const fe *b, fe *out, size_t count);
void diag_blake3_elems(hipStream_t st, const fe *in, int k, size_t count, uint8_t *out);
}  // namespace zk
