// kernels.hip -- gfx950 kernels of the STARK prove path (winterfell 0.9 generate_proof stages
// S2..S6; kernel list K1..K8 of SURVEY 7).
//
// Data layout in HBM (DESIGN.md "Data layout"):
//   * polynomials: one contiguous array of n coefficients per column;
//   * LDE values:  coset-major per column, element (c, i) at base[(c*B + i%B)*n + i/B], i the
//     natural LDE index (x_i = 3 * w_N^i).  A coset is a plain size-n NTT output, rows i and
//     i + B (the evaluation frame) are neighbours, and 8 consecutive lanes of a wave reading
//     natural indices touch 8 cosets x 16 B, so every wave load covers whole 128-B lines.
//   * digests: 32-byte BLAKE3 words, leaves in natural order, nodes[1] = root.
// All arithmetic is exact f128 (f128.hpp); no floating point anywhere.
#include <hip/hip_runtime.h>
#include <bitset>
#include <mutex>
#include <stdlib.h>
#include <string.h>

#include "blake3.hpp"
#include "fri_small.hpp"
#include "rescue_consts.hpp"
#include "zk_internal.hpp"

namespace zk {

#define ZK_LAUNCH_CHECK() (void)hipGetLastError()

static inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

__device__ __forceinline__ fe ld_fe(const fe *p) { return *p; }
__device__ __forceinline__ void st_fe(fe *p, fe v) { *p = v; }

// w_n^t from split tables (t < n)
__device__ __forceinline__ fe pow_split(const fe *lo, const fe *hi, size_t t) {
    return fe_mul(lo[t & 2047], hi[t >> 11]);
}

// ================================================================ NTT engine
// One block owns a tile of TILE field elements in LDS = LPB lines of M = TILE / LPB elements.
// Each line is loaded in bit-reversed position and transformed in place by log2(M) radix-2
// decimation-in-time stages; the result is in natural order.  Lines are padded by one element
// so that LPB lanes writing the same position of consecutive lines hit different banks.
#ifndef ZK_NTT_THREADS
#define ZK_NTT_THREADS 1024
#endif
#ifndef ZK_NTT_TILE
#define ZK_NTT_TILE 4096
#endif
#ifndef ZK_NTT_WAVES
#define ZK_NTT_WAVES 8  // waves per SIMD: two 1024-thread blocks per CU (the LDS limit) need <= 64 VGPRs
#endif
constexpr int NTT_THREADS = ZK_NTT_THREADS;

#ifndef ZK_NTT_LAZY
#define ZK_NTT_LAZY 1  // fused UNI pass-1 rounds keep butterfly sums partially reduced (fe_add_lazy); the pass
#endif                 // twiddle multiply makes the stored values canonical (A/B: pass 1 -0.09 ms per proof)
#ifndef ZK_NTT_J0
#define ZK_NTT_J0 1  // plain-DFT wave-uniform rounds: the waves with j = 0 skip their three unit-twiddle multiplies
#endif
#ifndef ZK_NTT_SWZ
#define ZK_NTT_SWZ 1  // XOR-swizzled LDS tiles (0: one pad element per line)
#endif

// LDS layout of a tile: LPB lines of M = 2^LOGM elements (16 B, i.e. 4 banks, each).  With 64 banks a
// 16-lane quarter-wave is conflict-free when its elements differ in the low 4 index bits.
//   swizzled (M >= 64): element (line, pos) at line*M + (sw(pos) ^ ((line & LMASK) << R)), where
//   sw(x) = x ^ 5*((x >> 4) & 3) folds index bits 4-5 into bits 0-3 (the radix-4 rounds with h = 1 and
//   h = 4 stride through exactly those bits) and the line goes above the R = log2(16/LPB) bits that 16
//   lanes vary in the load and pass-2 store phases.  sw is linear over XOR, so an element at pos + d
//   (d's bits zero in pos) is idx ^ sw(d).
//   padded (small M): line*(M + 1) + pos.
//   The 1024-point / 4-line, 2048-point / 2-line and 4096-point / 1-line tiles (UNI below: the four-step passes)
//   fold bits 4-7, 8-9 and 10-11 into bits 0-3 instead: their rounds with h <= 16 give every wave one
//   butterfly index j (lanes spread over lines and groups, stride 4h), which the bits-4-5 fold leaves 4- and
//   16-way conflicted; this one is conflict-free for those, the other rounds, the load orders and the
//   stores (host model: tools/lds_bank_model.py).  Bits 2-3 are folded into bits 0-1 too, for the fused first round
//   (ZK_NTT_FUSE: lanes spread over 4 lines x 4 butterflies write one position each, 4-way conflicted without it).
template <int LOGM, int TILE>
struct Lds {
    static constexpr int M = 1 << LOGM, LPB = TILE >> LOGM;
    static constexpr bool SWZ = ZK_NTT_SWZ && LOGM >= 6;
    // 2048-point lines (the odd splits, 2^21 and 2^23) too: A/B pass 1 at 2^21 13.2 -> 12.3 ms, pass 2 at 2^23 51.8 ->
    // 49.1 ms per proof; their trailing radix-2 stage stays generic
    static constexpr bool UNI = (LOGM >= 10 && LOGM <= 12) && TILE == 4096 && NTT_THREADS == 1024;
    static constexpr int LLPB = LPB >= 16 ? 4 : LPB >= 8 ? 3 : LPB >= 4 ? 2 : LPB >= 2 ? 1 : 0;
    static constexpr int R = 4 - LLPB;
    static constexpr int LMASK = (1 << LLPB) - 1;
    __device__ __forceinline__ static int sw(int x) {
        if constexpr (UNI) return x ^ ((x >> 4) & 15) ^ ((x >> 8) & 3) ^ (((x >> 10) & 3) << 2) ^ ((x >> 2) & 3);
        return SWZ ? x ^ (((x >> 4) & 3) * 5) : x;
    }
    __device__ __forceinline__ static int idx(int line, int pos) {
        if constexpr (SWZ) return line * M + (sw(pos) ^ ((line & LMASK) << R));
        else return line * (M + (LOGM >= 4 ? 1 : 0)) + pos;
    }
    __device__ __forceinline__ static int at(int p, int d) {
        if constexpr (SWZ) return p ^ sw(d);
        else return p + d;
    }
    // load phase: the v-th element of a line (in lane order) is DFT input k = v rotated right by R bits,
    // so that after the bit reversal the R low lane bits land in the low position bits
    __device__ __forceinline__ static int load_k(int v) {
        if constexpr (SWZ && R > 0) return ((v & ((1 << R) - 1)) << (LOGM - R)) | (v >> R);
        else return v;
    }
    static constexpr size_t bytes() { return (size_t)(SWZ ? TILE : TILE + (LOGM >= 4 ? LPB : 0)) * sizeof(fe); }
};

// One radix-4 round (stages lg, lg+1), compile-time lg so every shift and mask is an immediate.
// CT (coset-table mode): tw is a per-line-set stage table, tw[h + j] = the stage twiddle for half-size h
// and butterfly index j (a DFT evaluated on a coset c<w_M>: c^(M/2h) w_2h^j), instead of w_4096 powers.
// UNI tiles, rounds with h <= 16: wave w takes butterfly index j = w / (16/h) for 1024/h (line, group)
// pairs, so its three twiddles are wave-uniform and multiply through their W sets (fe_mul_uniform, scalar
// loads from `ws`, the W-set table indexed exactly like `tw4096`).  Same butterflies, same values.
template <int LOGM, int TILE, int LG, bool CT, bool LZ = false>
__device__ __forceinline__ void r4_round(fe *s, const fe *tw4096, const fe_ws *ws, const fe_w2 *w2t) {
    constexpr int M = 1 << LOGM;
    constexpr int Q = TILE / 4;
    constexpr int h = 1 << (LG - 1);
    using L = Lds<LOGM, TILE>;
    // paired final reductions (f128.hpp ws_fold2) only where the sums are plain and canonical (pass 2 and the odd
    // splits): in the coset and lazy pass-1 rounds the pairs' extra live registers spill at the 64-VGPR budget
    // (tools/isa_census.py), and the A/B of profiles/r06b_ab_fold2.txt found no gain to pay for that
    constexpr bool F2 = !CT && !LZ;
    if constexpr (L::UNI && h <= 16) {
        constexpr int LH = LG - 1;
        const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), l = threadIdx.x & 63;
        const int j = w >> (4 - LH);
        const int pidx = ((w & ((16 >> LH) - 1)) << 6) | l;  // < 1024 / h: (line, group) pairs
        const int line = pidx >> (LOGM - 2 - LH), grp = pidx & ((M >> (2 + LH)) - 1);
        const int p = L::idx(line, grp * 4 * h + j), ph = L::at(p, h), p2h = L::at(p, 2 * h), p3h = L::at(p, 3 * h);
        const fe x0 = s[p], x1 = s[ph], x2 = s[p2h], x3 = s[p3h];
        // plain DFT, j = 0 (wave-uniform): w_2h^0 = w_4h^0 = 1, only w_4h^h = w_4 remains.  Under LZ the tile
        // holds lazy (< 2^128, not canonical) values and the skipped multiplies were what made the second
        // operands of the lazy add/sub canonical, so those waves canonicalise x1, x3 and a2 instead.
        const bool triv = !CT && ZK_NTT_J0 && j == 0;
        fe t1 = x1, t3 = x3;
        if (!triv) {
            const fe_ws W1 = load_fe_ws(ws, CT ? h + j : j << (12 - LG));
            mul_uniform_pair<F2>(x1, W1, x3, W1, t1, t3);
        } else if (LZ) {
            t1 = fe_canon(x1);
            t3 = fe_canon(x3);
        }
        fe a0, a1, a2, a3;
        addsub2<LZ>(x0, t1, x2, t3, a0, a1, a2, a3);
        fe u2 = a2, u3;
        if constexpr (F2) {
            const fe_ws W3 = load_fe_ws(ws, CT ? 3 * h + j : (j + h) << (11 - LG));
            if (!triv) {
                mul_uniform_pair<true>(a2, load_fe_ws(ws, CT ? 2 * h + j : j << (11 - LG)), a3, W3, u2, u3);
            } else {
                u3 = fe_mul_uniform(a3, W3);
            }
        } else {
            if (!triv) u2 = fe_mul_uniform(a2, load_fe_ws(ws, CT ? 2 * h + j : j << (11 - LG)));
            else if (LZ) u2 = fe_canon(a2);
            u3 = fe_mul_uniform(a3, load_fe_ws(ws, CT ? 3 * h + j : (j + h) << (11 - LG)));
        }
        fe o0, o1, o2, o3;
        addsub2<LZ>(a0, u2, a1, u3, o0, o2, o1, o3);
        s[p] = o0;
        s[p2h] = o2;
        s[ph] = o1;
        s[p3h] = o3;
        __syncthreads();
        return;
    }
    // (1024-point lines only: on the 2048- and 4096-point tiles of 2^21 .. 2^23 the same mapping measured no gain,
    // 51.4-51.6 vs 51.6-51.8 ms per 2^22 proof, device-resident 50.3-50.5 vs 50.1-50.3; profiles/r04_ab_grp2_2p22.txt)
    if constexpr (L::UNI && LOGM == 10 && h == 64) {
        // group-uniform twiddles (h = 64): wave w takes the 4 butterfly classes j = 4w .. 4w+3, one per quarter-wave,
        // each of the 16 (line, group) pairs a 4096-element tile holds (any M of a UNI tile), so the 16 lanes of a
        // quarter-wave share one twiddle and its W set (vector loads of one 64-B entry; fe_mul_wsv, 80 issue slots
        // against fe_mul_w2's 99).  The lanes of a quarter-wave differ in line and group: the UNI swizzle folds
        // both into the low 4 bits, so the LDS phases stay conflict-free.
        constexpr int LH = LG - 1;
        const int w = (int)threadIdx.x >> 6, l = threadIdx.x & 63;
        const int j = (w << 2) | (l >> 4);
        const int pidx = l & 15;
        const int line = pidx >> (LOGM - 2 - LH), grp = pidx & ((M >> (2 + LH)) - 1);
        const int p = L::idx(line, grp * 4 * h + j), ph = L::at(p, h), p2h = L::at(p, 2 * h), p3h = L::at(p, 3 * h);
        const fe_ws W1 = ws[CT ? h + j : j << (12 - LG)];
        const fe x0 = s[p], x1 = s[ph], x2 = s[p2h], x3 = s[p3h];
        fe t1, t3;
        mul_wsv_pair<F2>(x1, W1, x3, W1, t1, t3);
        fe a0, a1, a2, a3;
        addsub2<LZ>(x0, t1, x2, t3, a0, a1, a2, a3);
        fe u2, u3;
        mul_wsv_pair<F2>(a2, ws[CT ? 2 * h + j : j << (11 - LG)], a3, ws[CT ? 3 * h + j : (j + h) << (11 - LG)], u2, u3);
        fe o0, o1, o2, o3;
        addsub2<LZ>(a0, u2, a1, u3, o0, o2, o1, o3);
        s[p] = o0;
        s[p2h] = o2;
        s[ph] = o1;
        s[p3h] = o3;
        __syncthreads();
        return;
    }
    if constexpr (L::UNI) {
        // per-lane twiddles (h >= 64): the two-part form (fe_w2, 32 B per twiddle)
        const int q = threadIdx.x;
        const int line = q >> (LOGM - 2), local = q & (M / 4 - 1);
        const int j = local & (h - 1), grp = local >> (LG - 1);
        const int p = L::idx(line, grp * 4 * h + j), ph = L::at(p, h), p2h = L::at(p, 2 * h), p3h = L::at(p, 3 * h);
        const fe_w2 w1 = w2t[CT ? h + j : j << (12 - LG)];
        const fe x0 = s[p], x1 = s[ph], x2 = s[p2h], x3 = s[p3h];
        fe t1, t3;
        mul_w2_pair<F2>(x1, w1, x3, w1, t1, t3);
        fe a0, a1, a2, a3;
        addsub2<LZ>(x0, t1, x2, t3, a0, a1, a2, a3);
        fe u2, u3;
        mul_w2_pair<F2>(a2, w2t[CT ? 2 * h + j : j << (11 - LG)], a3, w2t[CT ? 3 * h + j : (j + h) << (11 - LG)], u2, u3);
        fe o0, o1, o2, o3;
        addsub2<LZ>(a0, u2, a1, u3, o0, o2, o1, o3);
        s[p] = o0;
        s[p2h] = o2;
        s[ph] = o1;
        s[p3h] = o3;
        __syncthreads();
        return;
    }
#pragma unroll
    for (int q = threadIdx.x; q < Q; q += NTT_THREADS) {
        const int line = q >> (LOGM - 2), local = q & (M / 4 - 1);
        const int j = local & (h - 1), grp = local >> (LG - 1);
        const int p = L::idx(line, grp * 4 * h + j), ph = L::at(p, h), p2h = L::at(p, 2 * h), p3h = L::at(p, 3 * h);
        const fe w1 = CT ? tw4096[h + j] : tw4096[j << (12 - LG)];
        const fe w2 = CT ? tw4096[2 * h + j] : tw4096[j << (11 - LG)];
        const fe w3 = CT ? tw4096[3 * h + j] : tw4096[(j + h) << (11 - LG)];
        const fe x0 = s[p], x1 = s[ph], x2 = s[p2h], x3 = s[p3h];
        const fe t1 = fe_mul(x1, w1), t3 = fe_mul(x3, w1);
        fe a0, a1, a2, a3;
        fe_addsub2(x0, t1, x2, t3, a0, a1, a2, a3);
        const fe u2 = fe_mul(a2, w2), u3 = fe_mul(a3, w3);
        fe o0, o1, o2, o3;
        fe_addsub2(a0, u2, a1, u3, o0, o2, o1, o3);
        s[p] = o0;
        s[p2h] = o2;
        s[ph] = o1;
        s[p3h] = o3;
    }
    __syncthreads();
}

// rounds LG, LG+2, ... while LG + 1 <= STOP, then (STOP = LOGM) the trailing radix-2 stage of an odd LOGM
template <int LOGM, int TILE, int LG, bool CT, int STOP = LOGM, bool LZ = false>
__device__ __forceinline__ void r4_rounds(fe *s, const fe *tw4096, const fe_ws *ws, const fe_w2 *w2t) {
    if constexpr (LG + 1 <= STOP) {
        r4_round<LOGM, TILE, LG, CT, LZ>(s, tw4096, ws, w2t);
        r4_rounds<LOGM, TILE, LG + 2, CT, STOP, LZ>(s, tw4096, ws, w2t);
    } else if constexpr (LG == LOGM && STOP == LOGM) {
        static_assert(!LZ, "lazy sums only in the fused UNI rounds");
        constexpr int M = 1 << LOGM;
        constexpr int half = 1 << (LG - 1);
        using L = Lds<LOGM, TILE>;
#pragma unroll
        for (int bf = threadIdx.x; bf < TILE / 2; bf += NTT_THREADS) {
            const int line = bf >> (LOGM - 1), local = bf & (M / 2 - 1);
            const int j = local & (half - 1), grp = local >> (LG - 1);
            const int i0 = L::idx(line, grp * 2 * half + j), i1 = L::at(i0, half);
            const fe w = CT ? tw4096[half + j] : tw4096[j << (12 - LG)];  // w_len^j = w_4096^(j * 4096/len)
            const fe u = s[i0];
            const fe v = fe_mul(s[i1], w);
            s[i0] = fe_add(u, v);
            s[i1] = fe_sub(u, v);
        }
        __syncthreads();
    }
}

// Radix-4 rounds: each radix-4 butterfly performs DIT stages lg and lg+1 (half h = 2^(lg-1)) on
// positions p0 + {0, h, 2h, 3h}, p0 = grp*4h + j, j < h:
//   stage lg   : (x0, x1), (x2, x3) with w_2h^j
//   stage lg+1 : (x0, x2) with w_4h^j, (x1, x3) with w_4h^(j+h)
// so a round reads and writes each LDS element once for two stages.  The first round (h = 1, j = 0)
// has w_2 = w_4^0 = 1 and needs a single multiply by w_4.  An odd log2(M) ends with one radix-2 stage.
// Inlined into each kernel: `s` stays an LDS pointer (ds_read/ds_write) and the twiddle table a
// global one (global_load, counted by vmcnt only; as a called function both were flat accesses
// and every LDS wait also waited for the twiddle loads).
// CT: coset-table mode (every round generic, the first one included: 4 multiplies per 4 points).
// ws: the W sets of tw4096 (same indexing), used by the rounds with wave-uniform twiddles (UNI tiles).
template <int LOGM, int TILE, bool CT = false>
__device__ __forceinline__ void lds_dft(fe *s, const fe *tw4096, const fe_ws *ws, const fe_w2 *w2t) {
    constexpr int M = 1 << LOGM;
    constexpr int Q = TILE / 4;
    if constexpr (CT) {
        r4_rounds<LOGM, TILE, 1, true>(s, tw4096, ws, w2t);
    } else if constexpr (LOGM >= 2) {
        using L = Lds<LOGM, TILE>;
        fe w4;
        fe_ws W4;
        if constexpr (L::UNI) W4 = load_fe_ws(ws, 1024);
        else w4 = tw4096[1024];
#pragma unroll
        for (int q = threadIdx.x; q < Q; q += NTT_THREADS) {
            const int line = q >> (LOGM - 2), local = q & (M / 4 - 1);
            const int p = L::idx(line, local * 4), p1 = L::at(p, 1), p2 = L::at(p, 2), p3 = L::at(p, 3);
            const fe x0 = s[p], x1 = s[p1], x2 = s[p2], x3 = s[p3];
            fe a0, a1, a2, d23, a3;
            fe_addsub2(x0, x1, x2, x3, a0, a1, a2, d23);
            if constexpr (L::UNI) a3 = fe_mul_uniform(d23, W4);
            else a3 = fe_mul(d23, w4);
            fe o0, o1, o2, o3;
            fe_addsub2(a0, a2, a1, a3, o0, o2, o1, o3);
            s[p] = o0;
            s[p2] = o2;
            s[p1] = o1;
            s[p3] = o3;
        }
        __syncthreads();
        r4_rounds<LOGM, TILE, 3, false>(s, tw4096, ws, w2t);
    } else {
        r4_rounds<LOGM, TILE, 1, false>(s, tw4096, ws, w2t);
    }
}

// ---- first and last radix-4 rounds fused with the tile's global load and store (ZK_NTT_FUSE, UNI tiles of
// 1024 threads, one butterfly per thread and round).  The first round's four inputs come straight from memory
// and the last round's four outputs go straight to memory, so a tile makes 4 LDS round trips and 4 block
// barriers for its 5 radix-4 rounds instead of 6 and 6, and a wave starts computing as soon as its own loads
// arrive.  Lanes take the line fastest (q % LPB), as the library's load and store phases do, so every wave
// access still covers 64-B row segments (LPB = 4) or 1-KiB runs (LPB = 1).
#ifndef ZK_NTT_FUSE
#define ZK_NTT_FUSE 1
#endif
template <int LOGM, int TILE>
struct Fuse {
    static constexpr bool OK = ZK_NTT_FUSE && Lds<LOGM, TILE>::UNI && TILE / 4 == NTT_THREADS;
    // odd LOGM (2048-point lines): the radix-4 rounds end one stage short, and the trailing radix-2 stage is the one
    // fused with the store (last_r2_to); every value stays canonical (no lazy sums)
    static constexpr bool ODD = LOGM % 2 == 1;
    static constexpr int STOP = ODD ? LOGM - 1 : LOGM - 2;  // r4_rounds bound before the fused last stage
    static constexpr bool LAZY = ZK_NTT_LAZY && !ODD;
};
// First round: thread q takes line q % LPB and the butterfly at bit-reversed positions 4g .. 4g+3 (g = q / LPB),
// i.e. DFT inputs k0 + {0, M/2, M/4, 3M/4} with k0 = brev(4g), fetched by load(line, k).  Plain: one multiply by
// w_4 (W set ws[1024]); CT (coset stage table): twiddles ws[1], ws[2], ws[3] as in r4_round<LG = 1, CT>.
template <int LOGM, int TILE, bool CT, bool LZ, typename Load>
__device__ __forceinline__ void first_round_from(fe *s, Load load, const fe_ws *ws) {
    using L = Lds<LOGM, TILE>;
    constexpr int M = 1 << LOGM, LPB = TILE / M;
    const int q = threadIdx.x, line = q % LPB, g = q / LPB;
    const int k0 = (int)(__brev((unsigned)(4 * g)) >> (32 - LOGM));
    const fe x0 = load(line, k0), x1 = load(line, k0 + M / 2), x2 = load(line, k0 + M / 4), x3 = load(line, k0 + 3 * M / 4);
    const int p = L::idx(line, 4 * g), p1 = L::at(p, 1), p2 = L::at(p, 2), p3 = L::at(p, 3);
    if constexpr (!CT) {
        const fe_ws W4 = load_fe_ws(ws, 1024);
        fe a0, a1, a2, d23;
        addsub2_v<LZ ? 2 : 0>(x0, x1, x2, x3, a0, a1, a2, d23);  // a2 is a second operand below: keep it canonical
        const fe a3 = fe_mul_uniform(d23, W4);
        fe o0, o1, o2, o3;
        addsub2<LZ>(a0, a2, a1, a3, o0, o2, o1, o3);
        s[p] = o0;
        s[p2] = o2;
        s[p1] = o1;
        s[p3] = o3;
    } else {
        const fe_ws W1 = load_fe_ws(ws, 1);
        fe t1, t3;
        mul_uniform_pair<false>(x1, W1, x3, W1, t1, t3);
        fe a0, a1, a2, a3;
        addsub2<LZ>(x0, t1, x2, t3, a0, a1, a2, a3);
        fe u2, u3;
        mul_uniform_pair<false>(a2, load_fe_ws(ws, 2), a3, load_fe_ws(ws, 3), u2, u3);
        fe o0, o1, o2, o3;
        addsub2<LZ>(a0, u2, a1, u3, o0, o2, o1, o3);
        s[p] = o0;
        s[p2] = o2;
        s[p1] = o1;
        s[p3] = o3;
    }
    __syncthreads();
}
// Last round (h = M/4): thread q takes line q % LPB and butterfly index j = q / LPB; its outputs at positions
// j + {0, h, 2h, 3h} go to store(line, pos, value).  Per-lane two-part twiddles as in r4_round's UNI branch.
template <int LOGM, int TILE, bool CT, bool LZ, typename Store>
__device__ __forceinline__ void last_round_to(const fe *s, const fe_ws *ws, const fe_w2 *w2t, Store store) {
    using L = Lds<LOGM, TILE>;
    constexpr int M = 1 << LOGM, LPB = TILE / M, LG = LOGM - 1, h = M / 4;
    const int q = threadIdx.x, line = q % LPB, j = q / LPB;
    const int p = L::idx(line, j), ph = L::at(p, h), p2h = L::at(p, 2 * h), p3h = L::at(p, 3 * h);
    const fe x0 = s[p], x1 = s[ph], x2 = s[p2h], x3 = s[p3h];
    fe t1, t3, u2, u3, a0, a1, a2, a3;
    // (W sets through vector loads for the 4 lanes of one j measured within noise: profiles/r04_ab_kernels_2p20.txt)
    const fe_w2 w1 = w2t[CT ? h + j : j << (12 - LG)];
    mul_w2_pair<!CT && !LZ>(x1, w1, x3, w1, t1, t3);
    addsub2<LZ>(x0, t1, x2, t3, a0, a1, a2, a3);
    mul_w2_pair<!CT && !LZ>(a2, w2t[CT ? 2 * h + j : j << (11 - LG)], a3, w2t[CT ? 3 * h + j : (j + h) << (11 - LG)], u2, u3);
    fe o0, o1, o2, o3;
    addsub2<LZ>(a0, u2, a1, u3, o0, o2, o1, o3);  // LZ: the store canonicalises (a multiply or fe_canon)
    store(line, j, o0);
    store(line, j + h, o1);
    store(line, j + 2 * h, o2);
    store(line, j + 3 * h, o3);
}

// Last stage of an odd LOGM (radix 2, h = M/2): thread q takes line q % LPB and butterflies j = q / LPB + k TILE/(2 LPB)
// ... over the TILE/2 butterflies; outputs j and j + h go to store(line, pos, value).  Per-lane two-part twiddles.
template <int LOGM, int TILE, bool CT, typename Store>
__device__ __forceinline__ void last_r2_to(const fe *s, const fe_w2 *w2t, Store store) {
    using L = Lds<LOGM, TILE>;
    constexpr int M = 1 << LOGM, LPB = TILE / M, h = M / 2;
#pragma unroll
    for (int bf = threadIdx.x; bf < TILE / 2; bf += NTT_THREADS) {
        const int line = bf % LPB, j = bf / LPB;
        const int i0 = L::idx(line, j), i1 = L::at(i0, h);
        const fe u = s[i0], v = fe_mul_w2(s[i1], w2t[CT ? h + j : j << (12 - LOGM)]);
        store(line, j, fe_add(u, v));
        store(line, j + h, fe_sub(u, v));
    }
}

// XCD-aware block order: the dispatcher deals consecutive workgroups round-robin to the 8 XCDs
// (separate L2s).  Neighbouring line groups share 128-B lines (each block reads 64-B row segments),
// so give XCD x the contiguous range [x*G/8, (x+1)*G/8) in dispatch order.  Needs G % 8 == 0.
__device__ __forceinline__ size_t xcd_block(size_t b, size_t G) {
    return (G & 7) ? b : (b & 7) * (G >> 3) + (b >> 3);
}

struct NttArgs {
    const fe *in;
    fe *out;
    size_t in_stride, out_stride;
    const fe *tw4096;             // DFT-stage table (forward or inverse)
    const fe_ws *tw_ws;           // ... its W sets (the wave-uniform rounds of UNI tiles)
    const fe_w2 *tw_w2;           // ... in two-part form (the per-lane rounds of UNI tiles)
    const fe *big_lo, *big_hi;    // w_n^t split tables (forward or inverse) for the inter-pass twiddle
    const fe *pre_lo, *pre_hi;    // optional pre-scale s^k (split table)
    const fe *pre_full;           // ... or the same from a full table (preferred when present)
    size_t pre_stride;            // coset r uses pre_full + r * pre_stride
    const fe *pass_tw;            // inter-pass twiddles [k1 * n2 + j2] (replaces big_lo/hi when present)
    fe post;                      // post-scale constant
    int has_post;
    int log_n;
    // batch entry b = column c * ncos + coset slot j (coset r = cos_r0 + j * cos_rstride): input column c at
    // in + c * in_stride, output at out + c * out_stride + j * out_jstride.  ncos = 1 for plain batches.
    int ncos, cos_r0, cos_rstride;
    size_t out_jstride;
    const fe *cos_stage;  // coset LDE (four-step): per-coset stage tables, 4096 apart (CosetTables::stage)
    const fe_ws *cos_stage_ws;  // ... their W sets
    const fe_w2 *cos_stage_w2;  // ... and two-part forms
    const fe *cos_pass;   // ... and per-coset pass-1 twiddles (s_r w_n^j2)^k1, n apart (CosetTables::pass)
    // Sparse columns (SparseCols): a column whose entries are zero but the last one transforms to last * fill
    // (fill: the transform of the unit vector e_(n-1); coset r's at fill + r * fill_stride).  Pass 1 skips its
    // blocks, pass 2 writes the product; nz[sp_col0 + column] == 0 marks such a column (four-step only)
    const unsigned *nz;
    const fe *sp_last, *sp_fill;
    size_t sp_fill_stride;
    int sp_col0;
    // fused detection (SparseCols::fused, interpolation pass 1): det[det_col0 + column] = 1 when an entry before the
    // last is nonzero, det[det_stride + ..] when one has 8 bits or more, det[2 det_stride + ..] when 32 or more
    unsigned *det;
    int det_col0, det_stride;
    int sp_all;  // (host) every batch entry is sparse: no transform, one fill pass (SparseCols::all, k_sparse_fill)
    // the AIR clock (SparseCols::idoff): column 0 found to hold 0 .. n-2 transforms to sp_id + (last - (n-1)) * fill
    const fe *sp_id;
    int sp_idoff;
    int sp_r0, sp_rshift;  // the fill tables' cosets: coset r at slot (r - sp_r0) >> sp_rshift (Plan::lde_slot)
    __device__ __forceinline__ bool sparse(uint32_t b) const {
        return nz && nz[sp_col0 + (int)(b / (uint32_t)ncos)] == 0;
    }
    __device__ __forceinline__ bool clock(uint32_t b) const {
        return nz && sp_idoff && sp_col0 + (int)(b / (uint32_t)ncos) == 0 && nz[sp_idoff] == 0;
    }
    // (32-bit: batch entries and grid sizes are < 2^32; 64-bit division is a long VALU sequence)
    __device__ __forceinline__ int coset_of(uint32_t b) const { return cos_r0 + (int)(b % (uint32_t)ncos) * cos_rstride; }
    __device__ __forceinline__ size_t fill_slot(uint32_t b) const { return (size_t)((coset_of(b) - sp_r0) >> sp_rshift); }
    __device__ __forceinline__ fe *out_of(uint32_t b) const {
        return out + (size_t)(b / (uint32_t)ncos) * out_stride + (size_t)(b % (uint32_t)ncos) * out_jstride;
    }
};

// Single pass: whole polynomial (n = M <= TILE) per line, LPB = TILE / n polys per block.
template <int LOGM, int TILE>
__global__ void __launch_bounds__(NTT_THREADS, ZK_NTT_WAVES) ntt_single(NttArgs a, int batch) {
    extern __shared__ fe s[];
    constexpr int M = 1 << LOGM;
    constexpr int LPB = TILE / M;
    const int b0 = blockIdx.x * LPB;
    for (int e = threadIdx.x; e < TILE; e += NTT_THREADS) {
        int line = e >> LOGM, k = e & (M - 1);
        int b = b0 + line;
        fe v = fe_zero();
        if (b < batch) {
            v = a.in[(size_t)(b / a.ncos) * a.in_stride + k];
            if (a.pre_full) v = fe_mul(v, a.pre_full[(size_t)a.coset_of(b) * a.pre_stride + k]);
            else if (a.pre_lo) v = fe_mul(v, pow_split(a.pre_lo, a.pre_hi, (size_t)k));
        }
        s[Lds<LOGM, TILE>::idx(line, (int)(__brev((unsigned)k) >> (32 - LOGM)))] = v;
    }
    __syncthreads();
    lds_dft<LOGM, TILE>(s, a.tw4096, a.tw_ws, a.tw_w2);
    for (int e = threadIdx.x; e < TILE; e += NTT_THREADS) {
        int line = e >> LOGM, j = e & (M - 1);
        int b = b0 + line;
        if (b >= batch) continue;
        fe v = s[Lds<LOGM, TILE>::idx(line, j)];
        if (a.has_post) v = fe_mul(v, a.post);
        a.out_of(b)[j] = v;
    }
}

// Four-step, pass 1.  n = n1 * n2, input index k = k1 + n1*k2.  A block takes LPB consecutive k1
// (lines of length n2 = 2^LOGM read at stride n1 -> LPB contiguous elements per row), runs the
// size-n2 DFT over k2, multiplies by w_n^(j2*k1) and writes X[k1*n2 + j2] (contiguous runs).
// Grid: one dimension over (line group, column), remapped per XCD: the 8/LPB line groups that share the
// input's 128-B lines fastest, then the column, so an XCD runs those line groups for every column back to
// back and its slice of the pass twiddle table stays in that XCD's L2 (columns outermost re-fetched the
// table once per column).
// CT (coset LDE): no input pre-scale -- the coset shift s_r^k = s_r^(k1) (s_r^n1)^(k2) is split into a DFT
// over the coset s_r^n1 <w_n2> (per-coset stage table, lds_dft<CT>: the first radix-4 round costs 4
// multiplies per 4 points instead of 1, the pre-scale's 4 are gone) and the line constant s_r^k1, folded
// into the per-coset pass twiddle (s_r w_n^j2)^k1.  Same outputs, 0.25 multiplies and one 16-B table read
// fewer per element.
// fused column detection (NttArgs::det): per-thread ORs of the entries a thread loads, flushed once per block
struct DetAcc {
    uint32_t any = 0, w8 = 0, w32 = 0;
    __device__ __forceinline__ void note(fe v) {
        const uint32_t h = (uint32_t)v.hi | (uint32_t)(v.hi >> 32) | (uint32_t)(v.lo >> 32);
        w32 |= h;
        w8 |= h | ((uint32_t)v.lo >> 8);
        any |= h | (uint32_t)v.lo;
    }
};
__device__ __forceinline__ void det_flush(const NttArgs &a, uint32_t b, const DetAcc &d) {
    const bool ba = __syncthreads_or(d.any != 0), b8 = __syncthreads_or(d.w8 != 0), b32 = __syncthreads_or(d.w32 != 0);
    if (threadIdx.x == 0) {
        const int c = a.det_col0 + (int)(b / (uint32_t)a.ncos);
        if (ba) a.det[c] = 1u;
        if (b8 && a.det_stride) a.det[a.det_stride + c] = 1u;
        if (b32 && a.det_stride) a.det[2 * a.det_stride + c] = 1u;
    }
}

template <int LOGM, int TILE, bool CT>
__global__ void __launch_bounds__(NTT_THREADS, ZK_NTT_WAVES) ntt_pass1(NttArgs a, int batch) {
    extern __shared__ fe s[];
    constexpr int M = 1 << LOGM;  // n2
    constexpr int LPB = TILE / M;
    const size_t n = (size_t)1 << a.log_n;
    const size_t n1 = n >> LOGM;
    const size_t lin = xcd_block(blockIdx.x, gridDim.x);
    const uint32_t lin32 = (uint32_t)lin;
    size_t k1_0;
    uint32_t b;
    // K1G line groups share the input's 128-B row segments (LPB elements of 16 B each) and are the fastest index, so
    // the blocks that read the same lines (and, in a coset LDE, the cosets of one column: consecutive batch
    // entries) run together on one XCD instead of `batch` blocks apart (A/B at 2^22, LPB = 1: pass 1 26.7 -> 24.8 ms
    // per proof; at 2^20, LPB = 4: 4.98 -> 4.86)
    constexpr uint32_t K1G = LPB >= 8 ? 1u : 8u / LPB;
    if (K1G > 1 && ((n1 / LPB) % K1G) == 0) {
        const uint32_t rest = lin32 / K1G;
        b = rest % (uint32_t)batch;
        k1_0 = (size_t)((rest / (uint32_t)batch) * K1G + lin32 % K1G) * LPB;
    } else {
        k1_0 = (size_t)(lin32 / (uint32_t)batch) * LPB;
        b = lin32 % (uint32_t)batch;
    }
    if (a.sparse(b) || a.clock(b)) return;  // pass 2 writes its output
    const fe *in = a.in + (size_t)(b / (uint32_t)a.ncos) * a.in_stride;
    const int r = a.coset_of(b);
    fe *out = a.out + b * a.out_stride;
    if constexpr (Fuse<LOGM, TILE>::OK) {
      // (the plain form only without an input pre-scale and with a pass-twiddle table, as ntt() sets it up)
      if (CT || (!a.pre_full && !a.pre_lo && a.pass_tw)) {
        const fe *stage = CT ? a.cos_stage + (size_t)r * 4096 : a.tw4096;
        const fe_ws *stage_ws = CT ? a.cos_stage_ws + (size_t)r * 4096 : a.tw_ws;
        const fe_w2 *stage_w2 = CT ? a.cos_stage_w2 + (size_t)r * 4096 : a.tw_w2;
        using F = Fuse<LOGM, TILE>;
        if (!CT && a.det) {  // (uniform) the interpolation of a host trace: detection fused with the tile load
            DetAcc d;
            first_round_from<LOGM, TILE, CT, F::LAZY>(
                s, [&](int line, int k2) {
                    const size_t k = k1_0 + line + n1 * (size_t)k2;
                    const fe v = ld_fe(in + k);
                    if (k != n - 1) d.note(v);
                    return v;
                }, stage_ws);
            det_flush(a, b, d);
        } else {
            first_round_from<LOGM, TILE, CT, F::LAZY>(
                s, [&](int line, int k2) { return ld_fe(in + k1_0 + line + n1 * (size_t)k2); }, stage_ws);
        }
        r4_rounds<LOGM, TILE, 3, CT, F::STOP, F::LAZY>(s, stage, stage_ws, stage_w2);
        const fe *ptw = CT ? a.cos_pass + (size_t)r * n : a.pass_tw;
        auto store = [&](int line, int j2, fe v) {
            const size_t o = (k1_0 + line) * M + j2;
            out[o] = fe_mul(v, ptw[o]);  // inter-pass twiddle w^(j2 k1) (CT: (s_r w_n^j2)^k1), contiguous over the block
        };
        if constexpr (F::ODD) last_r2_to<LOGM, TILE, CT>(s, stage_w2, store);
        else last_round_to<LOGM, TILE, CT, F::LAZY>(s, stage_ws, stage_w2, store);
        return;
      }
    }
    DetAcc d;
    for (int e = threadIdx.x; e < TILE; e += NTT_THREADS) {
        int line = e % LPB, k2 = Lds<LOGM, TILE>::load_k(e / LPB);
        size_t k = k1_0 + line + n1 * (size_t)k2;
        fe v = ld_fe(in + k);
        if (!CT && a.det && k != n - 1) d.note(v);
        if (!CT) {
            if (a.pre_full) v = fe_mul(v, a.pre_full[(size_t)r * a.pre_stride + k]);
            else if (a.pre_lo) v = fe_mul(v, pow_split(a.pre_lo, a.pre_hi, k));
        }
        s[Lds<LOGM, TILE>::idx(line, (int)(__brev((unsigned)k2) >> (32 - LOGM)))] = v;
    }
    __syncthreads();
    if (!CT && a.det) det_flush(a, b, d);
    if constexpr (CT)
        lds_dft<LOGM, TILE, true>(s, a.cos_stage + (size_t)r * 4096, a.cos_stage_ws + (size_t)r * 4096, a.cos_stage_w2 + (size_t)r * 4096);
    else lds_dft<LOGM, TILE>(s, a.tw4096, a.tw_ws, a.tw_w2);
    for (int e = threadIdx.x; e < TILE; e += NTT_THREADS) {
        int line = e >> LOGM, j2 = e & (M - 1);
        size_t k1 = k1_0 + line;
        fe v = s[Lds<LOGM, TILE>::idx(line, j2)];
        if (CT) {
            v = fe_mul(v, a.cos_pass[(size_t)r * n + k1_0 * M + e]);
        } else if (a.pass_tw) {
            v = fe_mul(v, a.pass_tw[k1_0 * M + e]);  // = w^(j2 k1), contiguous over the block
        } else {
            size_t t = ((size_t)j2 * k1) & (n - 1);
            v = fe_mul(v, pow_split(a.big_lo, a.big_hi, t));
        }
        out[k1 * M + j2] = v;
    }
}

// Four-step, pass 2.  Lines over k1 (length n1 = 2^LOGM, stride n2) for LPB consecutive j2;
// output A[n2*j1 + j2] (LPB contiguous per j1).
template <int LOGM, int TILE>
__global__ void __launch_bounds__(NTT_THREADS, ZK_NTT_WAVES) ntt_pass2(NttArgs a) {
    extern __shared__ fe s[];
    constexpr int M = 1 << LOGM;  // n1
    constexpr int LPB = TILE / M;
    const size_t n = (size_t)1 << a.log_n;
    const size_t n2 = n >> LOGM;
    const size_t j2_0 = xcd_block(blockIdx.x, gridDim.x) * LPB;
    const size_t b = blockIdx.y;
    if (a.sparse((uint32_t)b)) {
        // last * (the transform of e_(n-1)) over this block's outputs
        const int col = a.sp_col0 + (int)(b / (uint32_t)a.ncos);
        const fe last = a.sp_last[col];
        const fe *fill = a.sp_fill + a.fill_slot((uint32_t)b) * a.sp_fill_stride;
        fe *out = a.out_of((uint32_t)b);
        for (int e = threadIdx.x; e < TILE; e += NTT_THREADS) {
            const size_t o = n2 * (size_t)(e / LPB) + j2_0 + (size_t)(e % LPB);
            out[o] = fe_mul(last, fill[o]);
        }
        return;
    }
    if (a.clock((uint32_t)b)) {
        // the identity column's transform + (last - (n-1)) * (the transform of e_(n-1))
        const fe d = fe_sub(a.sp_last[0], fe_make(n - 1));
        const size_t off = a.fill_slot((uint32_t)b) * a.sp_fill_stride;
        const fe *fill = a.sp_fill + off, *id = a.sp_id + off;
        fe *out = a.out_of((uint32_t)b);
        for (int e = threadIdx.x; e < TILE; e += NTT_THREADS) {
            const size_t o = n2 * (size_t)(e / LPB) + j2_0 + (size_t)(e % LPB);
            out[o] = fe_add(id[o], fe_mul(d, fill[o]));
        }
        return;
    }
    const fe *in = a.in + b * a.in_stride;
    if constexpr (Fuse<LOGM, TILE>::OK) {
        fe *out = a.out_of(b);
        using F = Fuse<LOGM, TILE>;
        first_round_from<LOGM, TILE, false, false>(
            s, [&](int line, int k1) { return in[(size_t)k1 * n2 + j2_0 + line]; }, a.tw_ws);
        r4_rounds<LOGM, TILE, 3, false, F::STOP, false>(s, a.tw4096, a.tw_ws, a.tw_w2);
        auto store = [&](int line, int j1, fe v) {
            if (a.has_post) v = fe_mul(v, a.post);
            out[n2 * (size_t)j1 + j2_0 + line] = v;
        };
        if constexpr (F::ODD) last_r2_to<LOGM, TILE, false>(s, a.tw_w2, store);
        else last_round_to<LOGM, TILE, false, false>(s, a.tw_ws, a.tw_w2, store);
        return;
    }
    for (int e = threadIdx.x; e < TILE; e += NTT_THREADS) {
        int line = e % LPB, k1 = Lds<LOGM, TILE>::load_k(e / LPB);
        fe v = in[(size_t)k1 * n2 + j2_0 + line];
        s[Lds<LOGM, TILE>::idx(line, (int)(__brev((unsigned)k1) >> (32 - LOGM)))] = v;
    }
    __syncthreads();
    lds_dft<LOGM, TILE>(s, a.tw4096, a.tw_ws, a.tw_w2);
    fe *out = a.out_of(b);
    for (int e = threadIdx.x; e < TILE; e += NTT_THREADS) {
        int line = e % LPB, j1 = e / LPB;
        fe v = s[Lds<LOGM, TILE>::idx(line, j1)];
        if (a.has_post) v = fe_mul(v, a.post);
        out[n2 * (size_t)j1 + j2_0 + line] = v;
    }
}

// Algorithmic operation counts of lds_dft per element (for the profiler): the first radix-4 round
// multiplies one of four elements, every further radix-4 round one per element, a trailing radix-2
// stage one per two; every stage adds or subtracts once per element.
static double dft_muls_per_elem(int logm) {
    if (logm < 2) return 0.5;
    return 0.25 + (double)((logm - 2) / 2) + ((logm & 1) ? 0.5 : 0.0);
}
// The profiler's multiply count is in fe_mul-equivalents, each kind priced at its issue cost relative to
// fe_mul's 113 slots (tools/ubench/fmul_lab.hip): a wave-uniform twiddle through its W set 80 (UNI rounds
// h = 1, 4, 16: 2.25 multiplies per element in the plain form, whose first round has one per four points,
// 3 in the coset-table form), a per-lane two-part twiddle 99 (the remaining LOGM/2 - 3 rounds).
static constexpr double ZK_UNIFORM_MUL_COST = 80.0 / 113.0, ZK_W2_MUL_COST = 99.0 / 113.0;
template <int LOGM, int TILE>
static double uniform_mul_discount(bool ct) {
    if (!Lds<LOGM, TILE>::UNI) return 0.0;
    return (ct ? 3.0 : 2.25) * (1.0 - ZK_UNIFORM_MUL_COST) + (LOGM / 2 - 3) * (1.0 - ZK_W2_MUL_COST);
}

template <int LOGM, int TILE>
static void launch_single(hipStream_t st, const NttArgs &a, int batch) {
    constexpr int LPB = TILE / (1 << LOGM);
    size_t sh = Lds<LOGM, TILE>::bytes();
    hipFuncSetAttribute((const void *)ntt_single<LOGM, TILE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    const double el = (double)batch * (1 << LOGM);
    ZK_PROF_OPS(st, "ntt_single", 32.0 * el,
                el * (dft_muls_per_elem(LOGM) - uniform_mul_discount<LOGM, TILE>(false) + (a.pre_full || a.pre_lo ? 1 : 0) + (a.has_post ? 1 : 0)),
                el * LOGM, hipLaunchKernelGGL((ntt_single<LOGM, TILE>), dim3(cdiv(batch, LPB)), dim3(NTT_THREADS), sh, st, a, batch));
}

template <int LOGM, int TILE>
static void launch_pass1(hipStream_t st, const NttArgs &a, int batch) {
    constexpr int LPB = TILE / (1 << LOGM);
    size_t n1 = ((size_t)1 << a.log_n) >> LOGM;
    size_t sh = Lds<LOGM, TILE>::bytes();
    const double el = (double)batch * ((size_t)1 << a.log_n);
    const dim3 grid(cdiv(n1, LPB) * batch);
    if (a.cos_stage) {
        hipFuncSetAttribute((const void *)ntt_pass1<LOGM, TILE, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
        ZK_PROF_OPS(st, "ntt_pass1", 32.0 * el, el * ((double)LOGM / 2.0 + 1.0 - uniform_mul_discount<LOGM, TILE>(true)), el * LOGM,
                    hipLaunchKernelGGL((ntt_pass1<LOGM, TILE, true>), grid, dim3(NTT_THREADS), sh, st, a, batch));
        return;
    }
    hipFuncSetAttribute((const void *)ntt_pass1<LOGM, TILE, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    ZK_PROF_OPS(st, "ntt_pass1", (a.pre_full ? 48.0 : 32.0) * el,
                el * (dft_muls_per_elem(LOGM) - uniform_mul_discount<LOGM, TILE>(false) + 1.0 + (a.pre_full || a.pre_lo ? 1 : 0) +
                      (a.pass_tw ? 0 : 1)),
                el * LOGM,
                hipLaunchKernelGGL((ntt_pass1<LOGM, TILE, false>), grid, dim3(NTT_THREADS), sh, st, a, batch));
}

template <int LOGM, int TILE>
static void launch_pass2(hipStream_t st, const NttArgs &a, int batch) {
    constexpr int LPB = TILE / (1 << LOGM);
    size_t n2 = ((size_t)1 << a.log_n) >> LOGM;
    size_t sh = Lds<LOGM, TILE>::bytes();
    hipFuncSetAttribute((const void *)ntt_pass2<LOGM, TILE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    const double el = (double)batch * ((size_t)1 << a.log_n);
    ZK_PROF_OPS(st, "ntt_pass2", 32.0 * el, el * (dft_muls_per_elem(LOGM) - uniform_mul_discount<LOGM, TILE>(false) + (a.has_post ? 1 : 0)),
                el * LOGM,
                hipLaunchKernelGGL((ntt_pass2<LOGM, TILE>), dim3(cdiv(n2, LPB), batch), dim3(NTT_THREADS), sh, st, a));
}

#define ZK_DISPATCH_LOGM(logm, FN, ...)           \
    switch (logm) {                               \
    case 1: FN<1, TILE>(__VA_ARGS__); break;      \
    case 2: FN<2, TILE>(__VA_ARGS__); break;      \
    case 3: FN<3, TILE>(__VA_ARGS__); break;      \
    case 4: FN<4, TILE>(__VA_ARGS__); break;      \
    case 5: FN<5, TILE>(__VA_ARGS__); break;      \
    case 6: FN<6, TILE>(__VA_ARGS__); break;      \
    case 7: FN<7, TILE>(__VA_ARGS__); break;      \
    case 8: FN<8, TILE>(__VA_ARGS__); break;      \
    case 9: FN<9, TILE>(__VA_ARGS__); break;      \
    case 10: FN<10, TILE>(__VA_ARGS__); break;    \
    case 11: FN<11, TILE>(__VA_ARGS__); break;    \
    case 12: FN<12, TILE>(__VA_ARGS__); break;    \
    default: break;                               \
    }

void ntt_run(hipStream_t st, const NttArgs &a, int batch, fe *tmp);

int ntt_log_n2(int L) {
    const int bal = (L + 1) / 2;
    if (L < 20) return bal;
    return std::min(12, L - 10);  // pass-2 lines of 1024 while pass-1 lines fit a 4096-element tile
}

void ntt(hipStream_t st, const NttTables &T, const fe *in, size_t in_stride, fe *out, size_t out_stride, int batch,
         bool inverse, const PowTable *pre, const fe *post_scale, fe *tmp, const SparseCols *sp) {
    NttArgs a;
    memset(&a, 0, sizeof a);
    a.in = in;
    a.out = out;
    a.in_stride = in_stride;
    a.out_stride = out_stride;
    a.tw4096 = inverse ? T.dft_inv : T.dft_fwd;
    a.tw_ws = inverse ? T.dft_inv_ws : T.dft_fwd_ws;
    a.tw_w2 = inverse ? T.dft_inv_w2 : T.dft_fwd_w2;
    a.big_lo = inverse ? T.inv_lo : T.fwd_lo;
    a.big_hi = inverse ? T.inv_hi : T.fwd_hi;
    a.pre_lo = pre ? pre->lo : nullptr;
    a.pre_hi = pre ? pre->hi : nullptr;
    a.pre_full = pre ? pre->full : nullptr;
    a.pre_stride = 0;
    a.pass_tw = inverse ? T.inv_pass : T.fwd_pass;  // inter-pass twiddles from a full table
    a.has_post = post_scale != nullptr;
    a.post = post_scale ? *post_scale : fe_zero();
    if (inverse && post_scale && T.log_n > 12 && T.inv_pass_n && fe_eq(*post_scale, T.inv_n)) {
        a.pass_tw = T.inv_pass_n;  // interpolation: n^-1 folded into the pass-1 twiddles
        a.has_post = 0;
    }
    a.log_n = T.log_n;
    a.ncos = 1;
    a.cos_r0 = 0;
    a.cos_rstride = 0;
    a.out_jstride = 0;
    a.cos_stage = a.cos_pass = nullptr;
    a.cos_stage_ws = nullptr;
    a.cos_stage_w2 = nullptr;
    if (sp && T.log_n > 12 && inverse && post_scale && fe_eq(*post_scale, T.inv_n)) {  // interpolation
        if (sp->fused) {
            a.det = const_cast<unsigned *>(sp->nz);
            a.det_col0 = sp->col0;
            a.det_stride = sp->wstride;
        } else {
            a.nz = sp->nz;
            a.sp_last = sp->last;
            a.sp_fill = sp->lagr;
            a.sp_fill_stride = 0;
            a.sp_col0 = sp->col0;
            a.sp_all = sp->all;
            a.sp_id = sp->id_poly;
            a.sp_idoff = sp->id_poly ? sp->idoff : 0;
        }
    }
    ntt_run(st, a, batch, tmp);
}

// Sparse columns the host knows of (SparseCols::all: the hinted columns of a host trace): the transform of column c
// is last[c] * fill (fill: the transform of e_(n-1), coset r's at fill + r * fill_stride), so one streaming pass reads
// each fill value once and writes it scaled into every column of the batch (instead of a pass-2 launch that re-read
// the fill per column: 32 B per output element -> 16 + 16 / ncols)
__global__ void __launch_bounds__(256) k_sparse_fill(NttArgs a, int ncols, int log_n) {
    const size_t n = (size_t)1 << log_n;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= ((size_t)a.ncos << log_n)) return;
    const uint32_t j = (uint32_t)(t >> log_n);
    const size_t k = t & (n - 1);
    const fe f = a.sp_fill[a.fill_slot(j) * a.sp_fill_stride + k];
    fe *o = a.out + (size_t)j * a.out_jstride + k;
    for (int c = 0; c < ncols; c++) o[(size_t)c * a.out_stride] = fe_mul(a.sp_last[a.sp_col0 + c], f);
}

// out[i] = F[i] + d * L[i], d wave-uniform (its W set a kernel argument): the clock column's coefficients / LDE from the
// identity column's and e_(n-1)'s (trace_lde_commit)
__global__ void __launch_bounds__(256) k_axpy_fill(const fe *F, const fe *L, fe_ws d, size_t cnt, fe *out) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < cnt) out[i] = fe_add(F[i], fe_mul_uniform(L[i], d));
}
void axpy_fill(hipStream_t st, const fe *F, const fe *L, const fe_ws &d, size_t cnt, fe *out) {
    ZK_PROF_OPS(st, "sparse_fill", 48.0 * cnt, (double)cnt, (double)cnt,
                hipLaunchKernelGGL(k_axpy_fill, dim3(cdiv(cnt, 256)), dim3(256), 0, st, F, L, d, cnt, out));
}

// the passes of one NTT call (single pass for n <= 4096, else four-step through tmp)
void ntt_run(hipStream_t st, const NttArgs &a, int batch, fe *tmp) {
    constexpr int TILE = ZK_NTT_TILE;
    const int L = a.log_n;
    if (a.nz && a.sp_all) {
        const int ncols = batch / a.ncos;
        const double pts = (double)a.ncos * (double)((size_t)1 << L);
        ZK_PROF_OPS(st, "sparse_fill", 16.0 * pts * (1 + ncols), pts * ncols, 0.0,
                    hipLaunchKernelGGL(k_sparse_fill, dim3(cdiv((size_t)a.ncos << L, 256)), dim3(256), 0, st, a, ncols, L));
        return;
    }
    if (L <= 12) {
        ZK_DISPATCH_LOGM(L, launch_single, st, a, batch);
        return;
    }
    // n = n1 * n2: pass-1 lines of n2 = 2^log_n2, pass-2 lines of n1 = 2^log_n1 (ntt_log_n2)
    const int log_n2 = ntt_log_n2(L), log_n1 = L - log_n2;
    NttArgs a1 = a;
    a1.out = tmp;
    a1.out_stride = (size_t)1 << L;
    a1.has_post = 0;
    ZK_DISPATCH_LOGM(log_n2, launch_pass1, st, a1, batch);
    NttArgs a2 = a;
    a2.in = tmp;
    a2.in_stride = (size_t)1 << L;
    a2.pre_lo = a2.pre_hi = a2.pre_full = nullptr;
    a2.cos_stage = a2.cos_pass = nullptr;
    a2.cos_stage_ws = nullptr;
    a2.cos_stage_w2 = nullptr;
    ZK_DISPATCH_LOGM(log_n1, launch_pass2, st, a2, batch);
}

void ntt_lde(hipStream_t st, const NttTables &T, const CosetTables &CT, const fe *in, size_t in_stride, int ncols,
             int r0, int rstride, int ncos, fe *out, size_t out_cstride, size_t out_jstride, fe *tmp,
             const SparseCols *sp) {
    NttArgs a;
    memset(&a, 0, sizeof a);
    a.in = in;
    a.out = out;
    a.in_stride = in_stride;
    a.out_stride = out_cstride;
    a.out_jstride = out_jstride;
    a.tw4096 = T.dft_fwd;
    a.tw_ws = T.dft_fwd_ws;
    a.tw_w2 = T.dft_fwd_w2;
    a.big_lo = T.fwd_lo;
    a.big_hi = T.fwd_hi;
    a.pass_tw = T.fwd_pass;
    a.log_n = T.log_n;
    a.ncos = ncos;
    a.cos_r0 = r0;
    a.cos_rstride = rstride;
    const size_t n = (size_t)1 << T.log_n;
    if (T.log_n <= 12) {  // single pass: pre-scale from the full (3 w_N^r)^k tables
        a.pre_full = CT.full;
        a.pre_stride = n;
    } else {
        a.cos_stage = CT.stage;
        a.cos_stage_ws = CT.stage_ws;
        a.cos_stage_w2 = CT.stage_w2;
        a.cos_pass = CT.pass;
        if (sp && !sp->fused) {
            a.nz = sp->nz;
            a.sp_last = sp->last;
            a.sp_fill = sp->lagr_lde;
            a.sp_fill_stride = n;
            a.sp_col0 = sp->col0;
            a.sp_all = sp->all;
            a.sp_id = sp->id_lde;
            a.sp_idoff = sp->id_lde ? sp->idoff : 0;
            a.sp_r0 = sp->lde_r0;
            a.sp_rshift = sp->lde_shift;
        }
    }
    // up to 8 cosets per launch (tmp holds ncols * 8 * n): every column of 8 cosets in one grid, so
    // one launch drain per pass instead of one per coset
    for (int j0 = 0; j0 < ncos; j0 += 8) {
        NttArgs b = a;
        b.ncos = std::min(8, ncos - j0);
        b.cos_r0 = r0 + j0 * rstride;
        b.out = out + (size_t)j0 * out_jstride;
        ntt_run(st, b, ncols * b.ncos, tmp);
    }
}

__global__ void k_pass_twiddles(const fe *lo, const fe *hi, int log_n, int log_n2, fe *out, fe *out_scaled, fe scale) {
    const size_t n = (size_t)1 << log_n;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < n; idx += (size_t)gridDim.x * blockDim.x) {
        const size_t k1 = idx >> log_n2, j2 = idx & (((size_t)1 << log_n2) - 1);
        const fe w = pow_split(lo, hi, (j2 * k1) & (n - 1));
        out[idx] = w;
        if (out_scaled) out_scaled[idx] = fe_mul(w, scale);
    }
}

// out[k1 * n2 + j2] = s^k1 * pass[k1 * n2 + j2]  (= (s w_n^j2)^k1): the per-coset pass-1 twiddles
__global__ void k_coset_pass(const fe *lo, const fe *hi, const fe *pass, int log_n, int log_n2, fe *out) {
    const size_t n = (size_t)1 << log_n;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < n; idx += (size_t)gridDim.x * blockDim.x)
        out[idx] = fe_mul(pow_split(lo, hi, idx >> log_n2), pass[idx]);
}

void coset_pass_tables(hipStream_t st, const fe *s_lo, const fe *s_hi, const fe *fwd_pass, int log_n, int log_n2,
                       fe *out) {
    const size_t n = (size_t)1 << log_n;
    hipLaunchKernelGGL(k_coset_pass, dim3(std::min<size_t>(cdiv(n, 256), 65536)), dim3(256), 0, st, s_lo, s_hi, fwd_pass,
                       log_n, log_n2, out);
}

void make_pass_twiddles(hipStream_t st, NttTables &T) {
    const size_t n = (size_t)1 << T.log_n;
    const int log_n2 = ntt_log_n2(T.log_n);  // pass-1 line length, as in ntt_run()
    const unsigned blocks = std::min<size_t>(cdiv(n, 256), 65536);
    hipLaunchKernelGGL(k_pass_twiddles, dim3(blocks), dim3(256), 0, st, T.fwd_lo, T.fwd_hi, T.log_n, log_n2, T.fwd_pass,
                       (fe *)nullptr, fe_zero());
    hipLaunchKernelGGL(k_pass_twiddles, dim3(blocks), dim3(256), 0, st, T.inv_lo, T.inv_hi, T.log_n, log_n2, T.inv_pass,
                       T.inv_pass_n, T.inv_n);
}

__global__ void k_pow_expand(const fe *lo, const fe *hi, size_t n, fe *out) {
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n; t += (size_t)gridDim.x * blockDim.x)
        out[t] = pow_split(lo, hi, t);
}

void pow_expand(hipStream_t st, const fe *lo, const fe *hi, size_t n, fe *out) {
    hipLaunchKernelGGL(k_pow_expand, dim3(std::min<size_t>(cdiv(n, 256), 65536)), dim3(256), 0, st, lo, hi, n, out);
}

// ================================================================ grinding (proof of work)
// nonce candidates start .. start+count: BLAKE3(seed || nonce_le64) (one 40-byte block) whose first
// u64 has >= bits trailing zeros; the smallest such nonce wins (winterfell searches from 1 upward).
__global__ void k_grind(const uint32_t *seed, uint64_t start, uint32_t count, int bits, unsigned long long *best) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const uint64_t nonce = start + t;
    uint32_t m[16], cv[8];
#pragma unroll
    for (int i = 0; i < 8; i++) m[i] = seed[i];
    m[8] = (uint32_t)nonce;
    m[9] = (uint32_t)(nonce >> 32);
#pragma unroll
    for (int i = 10; i < 16; i++) m[i] = 0;
    b3::iv(cv);
    b3::compress(cv, m, 0, 0, 40, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT);
    const uint64_t head = (uint64_t)cv[0] | ((uint64_t)cv[1] << 32);
    const int tz = head ? __builtin_ctzll(head) : 64;
    if (tz >= bits) atomicMin(best, (unsigned long long)nonce);
}

void grind_launch(hipStream_t st, const uint32_t *seed_dev, uint64_t start, uint32_t count, int bits,
                  unsigned long long *best_dev) {
    ZK_PROF(st, "grind", 0.0, hipLaunchKernelGGL(k_grind, dim3(cdiv(count, 256)), dim3(256), 0, st, seed_dev, start, count, bits, best_dev));
}

// ================================================================ hashing and Merkle trees
__device__ __forceinline__ void store_digest(uint8_t *dst, const uint32_t h[8]) {
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    d[0] = make_uint4(h[0], h[1], h[2], h[3]);
    d[1] = make_uint4(h[4], h[5], h[6], h[7]);
}
__device__ __forceinline__ void load_digest(const uint8_t *src, uint32_t h[8]) {
    const uint4 *s = reinterpret_cast<const uint4 *>(src);
    uint4 a = s[0], b = s[1];
    h[0] = a.x; h[1] = a.y; h[2] = a.z; h[3] = a.w;
    h[4] = b.x; h[5] = b.y; h[6] = b.z; h[7] = b.w;
}

// Leaf digests of coset-major LDE rows, one thread per row (K3/K5 of SURVEY 7): the rows i = 8q + r of the
// 2^log_rc cosets r0 <= r < r0 + 2^log_rc (all of them: r0 = 0, log_rc = log_b), leaves in natural order.
// (Fusing the bottom Merkle levels into this kernel was measured: the merges are compute-bound either way
// and the fused form lost.)
__global__ void __launch_bounds__(256) k_hash_rows(const fe *base, int ncols, int log_n, int log_b, int r0, int log_rc,
                                                   uint8_t *leaves) {
    const size_t M = (size_t)1 << (log_n + log_rc);
    const size_t n = (size_t)1 << log_n;
    const size_t B = (size_t)1 << log_b;
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < M; t += (size_t)gridDim.x * blockDim.x) {
        const size_t r = r0 + (t & (((size_t)1 << log_rc) - 1)), q = t >> log_rc;
        const fe *p = base + r * n + q;
        const size_t cstride = B * n;
        uint32_t h[8];
        b3::hash_elements(ncols, [&](int c) { return p[(size_t)c * cstride]; }, h);
        store_digest(leaves + 32 * ((q << log_b) + r), h);
    }
}

void hash_rows_cosets(hipStream_t st, const fe *base, int ncols, int log_n, int log_b, int r0, int log_rc,
                      uint8_t *leaves) {
    const size_t M = (size_t)1 << (log_n + log_rc);
    ZK_PROF(st, "hash_rows", (16.0 * ncols + 32) * M,
            hipLaunchKernelGGL(k_hash_rows, dim3(cdiv(M, 256)), dim3(256), 0, st, base, ncols, log_n, log_b, r0, log_rc, leaves));
}

// BLAKE3 blocks b0 .. b1 - 1 of every row: columns 4 b .. 4 b + 3 (64 bytes) compressed into the row's chaining
// value, kept in its leaf slot between launches (IV before block 0; after the last block the slot holds the digest).
// The trace rows (28 elements = 7 full blocks) are hashed this way as their columns' LDEs complete, so a
// host-resident proof hashes its rows under the rest of the upload instead of after it.
__global__ void __launch_bounds__(256) k_hash_rows_blocks(const fe *base, int log_n, int log_b, int b0, int b1, int nblk,
                                                          uint8_t *cv_leaves, VirtCols virt) {
    const size_t N = (size_t)1 << (log_n + log_b), n = (size_t)1 << log_n, B = (size_t)1 << log_b;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= N) return;
    const size_t r = t & (B - 1), q = t >> log_b;
    uint32_t h[8], m[16];
    uint8_t *slot = cv_leaves + 32 * ((q << log_b) + r);
    if (b0 == 0) b3::iv(h);
    else load_digest(slot, h);
    const uint32_t vmask = virt.mask >> (4 * b0) << (4 * b0) & ((b1 >= 8 ? 0u : 1u << (4 * b1)) - 1u);
    const fe lg = vmask ? virt.lagr_lde[r * n + q] : fe_zero();  // e_(n-1)'s LDE at this row (virtual columns)
    for (int blk = b0; blk < b1; blk++) {
        const fe *p = base + r * n + q + (size_t)(4 * blk) * B * n;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int c = 4 * blk + e;
            const fe v = ((vmask >> c) & 1u) ? fe_mul(lg, virt.last[c]) : p[(size_t)e * B * n];
            m[4 * e + 0] = (uint32_t)v.lo;
            m[4 * e + 1] = (uint32_t)(v.lo >> 32);
            m[4 * e + 2] = (uint32_t)v.hi;
            m[4 * e + 3] = (uint32_t)(v.hi >> 32);
        }
        const uint32_t flags = (blk == 0 ? b3::CHUNK_START : 0u) | (blk == nblk - 1 ? (b3::CHUNK_END | b3::ROOT) : 0u);
        b3::compress(h, m, 0, 0, 64, flags);
    }
    store_digest(slot, h);
}

void hash_rows_blocks(hipStream_t st, const fe *base, int ncols, int log_n, int log_b, int b0, int b1, uint8_t *leaves,
                      VirtCols virt) {
    const size_t N = (size_t)1 << (log_n + log_b);
    ZK_PROF(st, "hash_rows", (64.0 * (b1 - b0) + (b0 ? 64.0 : 32.0)) * N,
            hipLaunchKernelGGL(k_hash_rows_blocks, dim3(cdiv(N, 256)), dim3(256), 0, st, base, log_n, log_b, b0, b1,
                               ncols / 4, leaves, virt));
}

// Sparse-column detection: nz[c0 + c] = 1 when column c has a nonzero entry before its last one; last[c0 + c] = its
// last entry; with wstride > 0 also the width flags of SparseCols.  One pass over the columns (16 B per element read);
// nz must be zeroed first.
__global__ void __launch_bounds__(256) k_sparse_detect(const fe *trace, size_t n, int c0, unsigned *nz, fe *last,
                                                       int wstride, int idoff, size_t blk0) {
    constexpr int PER = 16;  // independent loads per thread (unrolled: all in flight at once)
    const int c = blockIdx.y;
    const fe *col = trace + (size_t)(c0 + c) * n;
    const size_t base = (blk0 + blockIdx.x) * (size_t)(256 * PER) + threadIdx.x;
    uint64_t any = 0, w8 = 0, w32 = 0, nid = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const size_t i = base + (size_t)k * 256;
        if (i < n - 1) {
            const fe v = col[i];
            any |= v.lo | v.hi;
            w8 |= (v.lo >> 8) | v.hi;
            w32 |= (v.lo >> 32) | v.hi;
            nid |= (v.lo ^ (uint64_t)i) | v.hi;
        }
    }
    if (idoff && c0 + c == 0) {  // (block-uniform) the AIR clock check of column 0
        const bool b_nid = __syncthreads_or(nid != 0);
        if (b_nid && threadIdx.x == 0) nz[idoff] = 1u;
    }
    // one flag write per block that saw a nonzero entry (a plain store: every writer stores 1), not one atomic per
    // wave -- 4096 same-address atomics per 64 MiB column serialised at L2 (0.38 ms per proof)
    const bool b_any = __syncthreads_or(any != 0);
    if (wstride) {
        const bool b8 = __syncthreads_or(w8 != 0), b32 = __syncthreads_or(w32 != 0);
        if (threadIdx.x == 0) {
            if (b8) nz[wstride + c0 + c] = 1u;
            if (b32) nz[2 * wstride + c0 + c] = 1u;
        }
    }
    if (b_any && threadIdx.x == 0) nz[c0 + c] = 1u;
    if (blockIdx.x == 0 && threadIdx.x == 0) last[c0 + c] = col[n - 1];
}

void sparse_detect(hipStream_t st, const fe *trace, size_t n, int c0, int nc, const SparseCols &sp) {
    sparse_detect_rows(st, trace, n, c0, nc, sp, 0, n);
}
// rows [r0, r1) only (r0 a multiple of 4096; the last row's values are read by every call): a sharded rank's share of
// the detection, whose flags the ranks all-gather and OR (shard.hip)
void sparse_detect_rows(hipStream_t st, const fe *trace, size_t n, int c0, int nc, const SparseCols &sp, size_t r0,
                        size_t r1) {
    constexpr size_t BR = 256 * 16;
    ZK_PROF(st, "sparse_detect", 16.0 * (double)(r1 - r0) * nc,
            hipLaunchKernelGGL(k_sparse_detect, dim3(cdiv(r1 - r0, BR), nc), dim3(256), 0, st, trace, n, c0,
                               const_cast<unsigned *>(sp.nz), const_cast<fe *>(sp.last), sp.wstride,
                               sp.id_poly ? sp.idoff : 0, r0 / BR));
}

// Packed narrow columns -> field elements: grid (row blocks, column), 4 rows per thread
__global__ void __launch_bounds__(256) k_expand_narrow(const uint8_t *src, NarrowCols nc, size_t n, fe *trace) {
    const int k = blockIdx.y;
    fe *out = trace + (size_t)nc.col[k] * n;
    const uint8_t *in = src + nc.off[k];
    const size_t i0 = (blockIdx.x * (size_t)256 + threadIdx.x) * 4;
    if (i0 >= n) return;
    uint32_t v[4];
    if (nc.width[k] == 1) {
        const uint32_t w = *reinterpret_cast<const uint32_t *>(in + i0);  // rows i0 .. i0+3 (n is a multiple of 4)
#pragma unroll
        for (int e = 0; e < 4; e++) v[e] = (w >> (8 * e)) & 0xffu;
    } else {
        const uint4 w = *reinterpret_cast<const uint4 *>(in + 4 * i0);
        v[0] = w.x;
        v[1] = w.y;
        v[2] = w.z;
        v[3] = w.w;
    }
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const size_t i = i0 + e;
        out[i] = i == n - 1 ? nc.last[k] : fe{(uint64_t)v[e], 0};
    }
}

void expand_narrow(hipStream_t st, const uint8_t *src, const NarrowCols &nc, size_t n, fe *trace) {
    if (!nc.count) return;
    hipLaunchKernelGGL(k_expand_narrow, dim3(cdiv(n / 4, 256), nc.count), dim3(256), 0, st, src, nc, n, trace);
}

// Commit to coset-major rows: leaves + full Merkle tree (nodes[1] = root).
void commit_rows_coset_major(hipStream_t st, const fe *base, int ncols, int log_n, int log_b, uint8_t *leaves,
                             uint8_t *nodes) {
    const size_t N = (size_t)1 << (log_n + log_b);
    hash_rows_cosets(st, base, ncols, log_n, log_b, 0, log_b, leaves);
    merkle_tree(st, leaves, N, nodes);
}

// FRI layer element i (natural index) of a layer stored natural (FriLayout::lb = 0) or coset-major over
// 2^lb cosets of 2^lcn points (layer 0 is the DEEP LDE as the coset NTT writes it: no reordering pass)
__device__ __forceinline__ size_t fri_at(FriLayout f, size_t i) {
    return ((i & (((size_t)1 << f.lb) - 1)) << f.lcn) + (i >> f.lb);
}
FriLayout fri_layout(size_t L, int lb) {
    int lg = 0;
    while (((size_t)1 << lg) < L) lg++;
    return FriLayout{lb, lg - lb};
}

__global__ void __launch_bounds__(256) k_hash_fri_rows(const fe *layer, size_t L, int fold, FriLayout f, uint8_t *leaves) {
    const size_t rows = L / fold;
    for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < rows; r += (size_t)gridDim.x * blockDim.x) {
        uint32_t h[8];
        b3::hash_elements(fold, [&](int k) { return layer[fri_at(f, r + (size_t)k * rows)]; }, h);
        store_digest(leaves + 32 * r, h);
    }
}

void commit_fri_layer(hipStream_t st, const fe *layer, size_t L, int fold, uint8_t *leaves, uint8_t *nodes, int lb) {
    const size_t rows = L / fold;
    const FriLayout f = fri_layout(L, lb);
    ZK_PROF(st, "hash_fri_rows", 16.0 * L + 32.0 * rows, hipLaunchKernelGGL(k_hash_fri_rows, dim3(cdiv(rows, 256)), dim3(256), 0, st, layer, L, fold, f, leaves));
    merkle_tree(st, leaves, rows, nodes);
}

// Three Merkle levels per launch: thread t merges the 8 child digests src[8t .. 8t+8) into nodes[cnt + 4t .. +4),
// their pairs into nodes[cnt/2 + 2t .. +2) and those into nodes[cnt/4 + t] (seven compressions per thread: one per
// thread and level-launch left every wave a single dependent compression behind its loads).  The child loads are
// software-pipelined: a grid of a few waves per SIMD walks the groups, each thread loading its next group's 8
// children (into registers) before merging the current one.  With one group per thread every wave of a launch
// loaded at the same moment and then merged at the same moment, so the child fetch (the launch reads all 2^k leaf
// digests) was never hidden behind compute (A/B on one box: merkle 0.64 -> 0.55 ms per 2^20 proof with a grid cap
// of 1024 / 2048 / 4096 blocks).
constexpr unsigned MERKLE_PF_BLOCKS = 2048;  // grid cap: two rounds of four waves per SIMD on 256 CUs
// half `half` of group t: children 8t + 4 half .. + 4 (c: 8 uint4) -> two parents and their parent g
__device__ __forceinline__ void merge_half3(const uint4 c[8], uint8_t *nodes, size_t cnt, size_t t, int half,
                                            uint32_t g[8]) {
    uint32_t l[8], r[8], h0[8], h1[8];
    auto dig = [&](int k, uint32_t d[8]) {
        const uint4 a = c[2 * k], b = c[2 * k + 1];
        d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
        d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
    };
    const size_t c0 = 4 * t + 2 * half;
    dig(0, l);
    dig(1, r);
    b3::merge(l, r, h0);
    store_digest(nodes + 32 * (cnt + c0), h0);
    dig(2, l);
    dig(3, r);
    b3::merge(l, r, h1);
    store_digest(nodes + 32 * (cnt + c0 + 1), h1);
    b3::merge(h0, h1, g);
    store_digest(nodes + 32 * (cnt / 2 + 2 * t + half), g);
}
#ifndef ZK_MERKLE_WAVES
#define ZK_MERKLE_WAVES 4  // waves per SIMD the pipelined three-level kernel targets (A/B: merkle 0.56-0.58 ms per
                           // proof at 4, 0.60-0.62 at 5, 0.67 at 6: the pipelined loads need the registers)
#endif
__global__ void __launch_bounds__(256, ZK_MERKLE_WAVES) k_merge_level3_pf(const uint8_t *src, uint8_t *nodes, size_t cnt) {
    const size_t q = cnt / 4, stride = (size_t)gridDim.x * blockDim.x;
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    uint4 cur[8], nxt[8];
    if (t < q) {
#pragma unroll
        for (int k = 0; k < 8; k++) cur[k] = s4[16 * t + k];
    }
    while (t < q) {
        const size_t tn = t + stride;
        uint32_t g0[8], g1[8], h[8];
#pragma unroll
        for (int k = 0; k < 8; k++) nxt[k] = s4[16 * t + 8 + k];  // second half of this group
        merge_half3(cur, nodes, cnt, t, 0, g0);
#pragma unroll
        for (int k = 0; k < 8; k++) cur[k] = nxt[k];
        if (tn < q) {
#pragma unroll
            for (int k = 0; k < 8; k++) nxt[k] = s4[16 * tn + k];  // first half of the next group
        }
        merge_half3(cur, nodes, cnt, t, 1, g1);
        b3::merge(g0, g1, h);
        store_digest(nodes + 32 * (cnt / 4 + t), h);
#pragma unroll
        for (int k = 0; k < 8; k++) cur[k] = nxt[k];
        t = tn;
    }
}

// Up to log2(P) + 1 levels in one block of P = blockDim.x threads: thread t merges the children
// src[2(bP + t)], src[2(bP + t) + 1] into first-level parent bP + t, then the block halves its level in
// LDS with one compression per thread per level; every node goes to its heap position.  Used for the
// upper part of a tree, where the three-level kernel's seven dependent compressions per thread made
// each launch a latency chain (the whole tail of a 2^22-leaf tree: 88 -> ~40 us).
__global__ void __launch_bounds__(512) k_merge_block(const uint8_t *src, uint8_t *nodes, size_t cnt) {
    __shared__ uint32_t lvl[512][8];
    const size_t P = blockDim.x, t = threadIdx.x, base = blockIdx.x * P;
    {
        uint32_t l[8], r[8], h[8];
        load_digest(src + 64 * (base + t), l);
        load_digest(src + 64 * (base + t) + 32, r);
        b3::merge(l, r, h);
        store_digest(nodes + 32 * (cnt + base + t), h);
#pragma unroll
        for (int w = 0; w < 8; w++) lvl[t][w] = h[w];
    }
    __syncthreads();
    size_t c = cnt, width = P, off = base;
    while (width > 1) {
        c >>= 1;
        width >>= 1;
        off >>= 1;
        uint32_t h[8];
        const bool act = t < width;
        if (act) b3::merge(lvl[2 * t], lvl[2 * t + 1], h);
        __syncthreads();
        if (act) {
#pragma unroll
            for (int w = 0; w < 8; w++) lvl[t][w] = h[w];
            store_digest(nodes + 32 * (c + off + t), h);
        }
        __syncthreads();
    }
}

#ifndef ZK_MERKLE_L3_MIN
#define ZK_MERKLE_L3_MIN 17  // log2 of the smallest level the three-level kernel takes (A/B: 17 > 20 > 16 > 14)
#endif
void merkle_tree(hipStream_t st, const uint8_t *leaves, size_t nl, uint8_t *nodes) {
    // invariant: src holds 2*cnt digests whose parents go to nodes[cnt .. 2cnt)
    size_t cnt = nl / 2;
    const uint8_t *src = leaves;
    // wide levels: three per launch, seven compressions per thread (throughput)
    while (cnt >= ((size_t)1 << ZK_MERKLE_L3_MIN)) {
        const unsigned blocks = std::min<unsigned>(cdiv(cnt / 4, 256), MERKLE_PF_BLOCKS);
        ZK_PROF(st, "merkle_level", 64.0 * cnt + 32.0 * (cnt + cnt / 2 + cnt / 4),
                hipLaunchKernelGGL(k_merge_level3_pf, dim3(blocks), dim3(256), 0, st, src, nodes, cnt));
        src = nodes + 32 * (cnt / 4);
        cnt /= 8;
    }
    // upper part: up to 10 levels per launch, one compression per thread per level (latency)
    while (cnt >= 1) {
        const size_t P = std::min<size_t>(512, cnt), roots = cnt / P;
        ZK_PROF(st, roots > 1 ? "merkle_level" : "merkle_top", 96.0 * 2 * cnt,
                hipLaunchKernelGGL(k_merge_block, dim3((unsigned)roots), dim3((unsigned)P), 0, st, src, nodes, cnt));
        if (roots == 1) break;
        src = nodes + 32 * roots;
        cnt = roots / 2;
    }
}

__global__ void k_gather_digests(const uint8_t *src, const uint64_t *idx, size_t k, uint8_t *out) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t < k) {
        uint32_t h[8];
        load_digest(src + 32 * idx[t], h);
        store_digest(out + 32 * t, h);
    }
}

void gather_digests(hipStream_t st, const uint8_t *src, const uint64_t *idx, size_t k, uint8_t *out) {
    if (k) hipLaunchKernelGGL(k_gather_digests, dim3(cdiv(k, 64)), dim3(64), 0, st, src, idx, k, out);
}

__global__ void k_gather_rows(const fe *base, int ncols, int log_n, int log_b, const uint64_t *pos, size_t k,
                              fe *out) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t < k * ncols) {
        size_t q = t / ncols, c = t % ncols;
        size_t i = pos[q], n = (size_t)1 << log_n, B = (size_t)1 << log_b;
        out[t] = base[(c * B + (i & (B - 1))) * n + (i >> log_b)];
    }
}

void gather_rows(hipStream_t st, const fe *base, int ncols, int log_n, int log_b, const uint64_t *pos, size_t k,
                 fe *out) {
    if (k) hipLaunchKernelGGL(k_gather_rows, dim3(cdiv(k * ncols, 64)), dim3(64), 0, st, base, ncols, log_n, log_b, pos,
                              k, out);
}

// ================================================================ batch inversion
// out[i] = 1 / ((x_i - a)(x_i - b)), x_i = xr[i & (B-1)] * w_n^(i >> log_b), via Montgomery's trick
// over K elements per thread (strided by the grid so every store is coalesced).
// Montgomery's trick over INV_K elements per thread (strided by the thread count T for coalescing):
// the running products are parked in `out` itself, so K can be large (one inversion per 64 elements)
// without holding them in registers.
#ifndef ZK_INV_K
#define ZK_INV_K 64
#endif
constexpr int INV_K = ZK_INV_K;

__device__ __forceinline__ fe inv_pair_denominator(const fe *xr, const fe *wlo, const fe *whi, size_t i, int log_n,
                                                   fe a, fe b) {
    const fe x = fe_mul(xr[i >> log_n], pow_split(wlo, whi, i & (((size_t)1 << log_n) - 1)));
    return fe_mul(fe_sub(x, a), fe_sub(x, b));
}

__global__ void __launch_bounds__(256) k_batch_inv_pairs(const fe *xr, int log_b, int log_n, const fe *wlo,
                                                         const fe *whi, fe a, fe b, fe *out, size_t total_threads) {
    const size_t N = (size_t)1 << (log_n + log_b);
    const size_t T = total_threads;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= T) return;
    fe acc = fe_one();
#pragma unroll 4
    for (int k = 0; k < INV_K; k++) {
        const size_t i = t + (size_t)k * T;  // coset-major: coset i >> log_n, position i % n
        if (i < N) {
            acc = fe_mul(acc, inv_pair_denominator(xr, wlo, whi, i, log_n, a, b));
            out[i] = acc;
        }
    }
    fe inv = fe_inv(acc);
#pragma unroll 4
    for (int k = INV_K - 1; k >= 0; k--) {
        const size_t i = t + (size_t)k * T;
        if (i >= N) continue;
        const fe d = inv_pair_denominator(xr, wlo, whi, i, log_n, a, b);
        out[i] = k > 0 ? fe_mul(inv, out[i - T]) : inv;
        inv = fe_mul(inv, d);
    }
}

void batch_inv_pairs(hipStream_t st, const NttTables &Tn, const fe *xr, int log_b, int log_n, fe a, fe b, fe *out) {
    size_t N = (size_t)1 << (log_n + log_b);
    size_t threads = (N + INV_K - 1) / INV_K;
    ZK_PROF(st, "batch_inv", 16.0 * N, hipLaunchKernelGGL(k_batch_inv_pairs, dim3(cdiv(threads, 256)), dim3(256), 0, st, xr, log_b,
                                                log_n, Tn.fwd_lo, Tn.fwd_hi, a, b, out, threads));
}

// Per-row divisor factors of the composition (once per plan: they depend only on the domain point x).
// In place over the 1/((x - 1)(x - g2)) table that batch_inv_pairs wrote to plane 0:
//   plane 0: (x - g2)(x - g1) / (x^n - 1)  transition divisor with the two exemptions, inverted
//   plane 1: 1 / (x - 1)                    step-0 assertions
//   plane 2: 1 / (x - g2)                   step-(n-2) assertions
__global__ void __launch_bounds__(256) k_divisor_tables(const fe *xr, int log_n, size_t P, const fe *wlo, const fe *whi,
                                                        fe g1, fe g2, Fe8 inv_zn, fe *out) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < P; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i >> log_n;
        const fe x = fe_mul(xr[r], pow_split(wlo, whi, i & (((size_t)1 << log_n) - 1)));
        const fe ibd = out[i], xa = fe_sub(x, g2), x1 = fe_sub(x, fe_one());
        out[i] = fe_mul(fe_mul(xa, fe_sub(x, g1)), inv_zn.v[r]);
        out[P + i] = fe_mul(xa, ibd);
        out[2 * P + i] = fe_mul(x1, ibd);
    }
}

void divisor_tables(hipStream_t st, const NttTables &Tn, const fe *xr, int log_cos, int log_n, fe g1, fe g2,
                    const Fe8 &inv_zn, fe *out) {
    batch_inv_pairs(st, Tn, xr, log_cos, log_n, fe_one(), g2, out);
    const size_t P = (size_t)1 << (log_cos + log_n);
    ZK_PROF(st, "batch_inv", 64.0 * P, hipLaunchKernelGGL(k_divisor_tables, dim3(cdiv(P, 256)), dim3(256), 0, st, xr,
                                                           log_n, P, Tn.fwd_lo, Tn.fwd_hi, g1, g2, inv_zn, out));
}

// ================================================================ constraint evaluation (K3)
// ProcessorAir::evaluate_transition (air/src/lib.rs:104-168, constrains.rs:95-216, flags.rs:37-91)
// fused with DefaultConstraintEvaluator's merge (sum of coeff * C_k), the transition divisor and the
// two boundary groups, one thread per CE-domain step.

__constant__ fe c_mds[16];

// Sequence the row loads of one section after the arithmetic of the previous one: the row pointer
// is laundered through an empty asm that consumes `dep`, so the scheduler cannot hoist ~45 independent
// loads to the top of the kernel (which by itself needs ~180 VGPRs and halves occupancy).
#define ZK_SEQ(ptr, dep) asm volatile("" : "+v"(ptr) : "v"(dep))

__device__ __forceinline__ fe cube(fe x) { return fe_mul(fe_mul(x, x), x); }

// Rescue MDS (crypto/src/rescue.rs:197-214) as signed small integers: row r = (-a, +b, -c, +d)
__device__ __forceinline__ fe mds_row(int r, const fe x[4]) {
    constexpr uint32_t M[16] = {729, 1080, 390, 40, 29160, 42471, 14520, 1210,
                                882090, 1277640, 429429, 33880, 24698520, 35708310, 11935560, 925771};
    acc160 pos = acc160_zero(), neg = acc160_zero();
    acc160_madd(neg, x[0], M[4 * r + 0]);
    acc160_madd(pos, x[1], M[4 * r + 1]);
    acc160_madd(neg, x[2], M[4 * r + 2]);
    acc160_madd(pos, x[3], M[4 * r + 3]);
    return fe_sub(acc160_reduce(pos), acc160_reduce(neg));
}

// Rescue inverse MDS through its adjugate (crypto/src/rescue.rs:197-233): INV_MDS = adj(MDS) / det with
// det = 3^24 and |adj| < 2^39 (every row signed + - + -; tests/test_oracle_core.py checks adj, det and the
// reference INV_MDS).  adj_row(r, y) = 3^24 (INV_MDS y)_r: four 128 x 39-bit products (8 MADs each) into a
// 192-bit accumulator and one reduction, instead of four full 128 x 128-bit products.
// s[0..6) += x * c, c < 2^40 (s stays below 2^192)
__device__ __forceinline__ void acc192_madd(uint32_t s[6], fe x, uint64_t c) {
    const uint32_t xs[4] = {lo32(x.lo), hi32(x.lo), lo32(x.hi), hi32(x.hi)};
    const uint32_t c0 = lo32(c), c1 = hi32(c);
    uint64_t t = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        t = (uint64_t)xs[k] * c0 + s[k] + (t >> 32);
        s[k] = lo32(t);
    }
    t = (uint64_t)s[4] + (t >> 32);
    s[4] = lo32(t);
    s[5] += hi32(t);
    t = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        t = (uint64_t)xs[k] * c1 + s[k + 1] + (t >> 32);
        s[k + 1] = lo32(t);
    }
    s[5] += hi32(t);
}
__device__ __forceinline__ fe adj_row(int r, const fe y[4]) {
    constexpr uint64_t A[16] = {491992666011ull, 234927627480ull, 26031357990ull, 666860040ull,
                                486140969160ull, 228216177189ull, 25147788120ull, 643043610ull,
                                468778791690ull, 208346129640ull, 22570830711ull, 573956280ull,
                                418414128120ull, 151093990710ull, 15496819560ull, 387420489ull};
    // pos starts at p 2^41 (> any sum of the negative terms), so pos - neg >= 0; both stay below 2^170
    uint32_t pos[6] = {0x0u, 0x200u, 0xffa60000u, 0xffffffffu, 0xffffffffu, 0x1ffu}, neg[6] = {0, 0, 0, 0, 0, 0};
    acc192_madd(pos, y[0], A[4 * r + 0]);
    acc192_madd(neg, y[1], A[4 * r + 1]);
    acc192_madd(pos, y[2], A[4 * r + 2]);
    acc192_madd(neg, y[3], A[4 * r + 3]);
    uint32_t d[6], b;
    d[0] = __builtin_subc(pos[0], neg[0], 0u, &b);
#pragma unroll
    for (int k = 1; k < 6; k++) d[k] = __builtin_subc(pos[k], neg[k], b, &b);
    return reduce_fold(d[0], d[1], d[2], d[3], d[4], d[5], 0u, 0u);
}
// 3^-72 mod p: the adjugate path's cubes carry 3^72, folded into the coefficients (ct3 = ct 3^-72)
static constexpr fe ZK_INV3_72 = fe{0x8092deb1ab776293ull, 0xf0185d00eca40a3bull};

// Block-shared constants of one evaluation (read through LDS so that none of them is pinned in
// SGPRs across the whole kernel -- the cause of SGPR spills and 1-wave occupancy before).
struct EvalShared {
    fe ct[20], cb[22], ct2[20], cb2[22];
    fe ct3[4], nct[4], ct3b[4], nctb[4];  // constraints 12..15: ct 3^-72 and -ct (planes a, b)
    fe delta, bnd1, bnd1b;
};

#ifndef ZK_EVAL_LAZY
#define ZK_EVAL_LAZY 1  // lazy 288-bit sum over the selector section's terms (base field)
#endif
#ifndef ZK_EVAL_WAVES
#define ZK_EVAL_WAVES 4  // waves per SIMD the register budget targets (measured: 4 > 3 > 1; the LDS stash also caps a CU at 4 blocks)
#endif
#ifndef ZK_EVAL_WAVES_EXT
#define ZK_EVAL_WAVES_EXT 4  // the two-plane (quadratic extension) variant (4: 110 VGPRs, no spills since the limb sums)
#endif
// KE coefficient planes: KE = 2 for FieldExtension::Quadratic, where the composition coefficients are
// E values; the composition is linear in them, so each constraint value is folded into two
// accumulators (K = a components, K2 = b components) and two planes comp[t], comp[plane + t] are written.
// BND: evaluate the boundary (assertion) terms here.  The single-GPU prover passes false and adds them
// in coefficient form instead (boundary_poly_add); the plug point and the sharded prover pass true.
template <int KE, bool BND>
__global__ void __launch_bounds__(256, KE == 1 ? ZK_EVAL_WAVES : ZK_EVAL_WAVES_EXT) k_eval_constraints(const fe *lde, int log_n, EvalMap map, const fe *periodic,
                                                          const fe *divs, const AirConsts *K, const AirConsts *K2,
                                                          size_t plane, fe *comp) {
    __shared__ EvalShared S;
    // lane-private stash of the columns two sections read (the 5 opcode bits, sponge 7 and 8, next-row s0): an LDS
    // slot instead of a second global load, which missed L2 (PMC: 4.30 GB per launch without, 3.42 with, against
    // 3.52 GB algorithmic; profiles/r04_pmc_traffic_eval_stash.txt).  8 x 256 x 16 B = 32 KiB per block, so four
    // 256-thread blocks (16 waves, the register budget's 4 per SIMD) still fit a CU's 160 KiB
    __shared__ fe stash[8][256];
    const int tid = threadIdx.x;
    {
        // one LDS slot per thread, every range bounded on both sides
        const int t = threadIdx.x;
        if (t < 20) S.ct[t] = K->coeff_t[t];
        else if (t < 42) S.cb[t - 20] = K->coeff_b[t - 20];
        else if (t == 42) S.bnd1 = K->bnd1;
        else if (t == 43) S.bnd1b = KE == 2 ? K2->bnd1 : fe_zero();
        else if (t == 44) S.delta = K->delta;
        else if (t >= 80 && t < 84) {
            S.ct3[t - 80] = fe_mul(K->coeff_t[12 + t - 80], ZK_INV3_72);
            S.nct[t - 80] = fe_neg(K->coeff_t[12 + t - 80]);
        } else if (KE == 2 && t >= 84 && t < 88) {
            S.ct3b[t - 84] = fe_mul(K2->coeff_t[12 + t - 84], ZK_INV3_72);
            S.nctb[t - 84] = fe_neg(K2->coeff_t[12 + t - 84]);
        }
        else if (KE == 2 && t >= 128 && t < 148) S.ct2[t - 128] = K2->coeff_t[t - 128];
        else if (KE == 2 && t >= 148 && t < 170) S.cb2[t - 148] = K2->coeff_b[t - 148];
        __syncthreads();
    }
    const int L = K->lwe_size;
    const size_t n = (size_t)1 << log_n;
    const size_t CE = n * map.nce;
    // thread t -> local CE coset jl = t / n, position q = t % n (a wave reads 64 consecutive positions of
    // one coset).  Global CE coset rc = ce0 + cestep * jl; CE step i = rc + 8q; its LDE rows sit in local
    // LDE coset slot jl << lshift at the same position.
    const size_t t_id = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t_id >= CE) return;
    const size_t jl = t_id >> log_n, q = t_id & (n - 1), qn = (q + 1) & (n - 1);
    const size_t rc = map.ce0 + map.cestep * jl;
    const size_t i = rc + 8 * q;
    const size_t r = jl << map.lshift;
    const fe *cb = lde + r * n;  // laundered by ZK_SEQ between sections
    const size_t cs = (size_t)map.lde_cosets * n;
#define CUR(c) cb[(size_t)(c)*cs + q]
#define NXT(c) cb[(size_t)(c)*cs + qn]
    const fe one = fe_one();
    const fe s0n = NXT(12);
    stash[5][tid] = s0n;
    fe t = fe_zero();  // sum of coeff_t[k] * C_k (kept reduced: a lazy 288-bit sum here costs 130 spills)
    fe t2 = fe_zero();  // the b-plane sum (KE = 2)
#define ZK_ACC(k, val)                                                    \
    do {                                                                  \
        const fe v_ = (val);                                              \
        t = fe_add(t, fe_mul(S.ct[k], v_));                               \
        if (KE == 2) {                                                    \
            t2 = fe_add(t2, fe_mul(S.ct2[k], v_));                        \
            asm volatile("" : "+v"(t2.lo), "+v"(t2.hi));                  \
        }                                                                 \
    } while (0)
    // 12..19 Rescue round / copy (constrains.rs:182-216) first: it needs only the opcode value and
    // is_push from the flags, so the ten selectors below are never live across it.
    {
        const fe b0 = CUR(5), b1 = CUR(4), b2 = CUR(3), b3 = CUR(2), b4 = CUR(1);
        stash[0][tid] = b0;
        stash[1][tid] = b1;
        stash[2][tid] = b2;
        stash[3][tid] = b3;
        stash[4][tid] = b4;
        // opcode = 16 b0 + 8 b1 + 4 b2 + 2 b3 + b4  (Horner by doubling: bits are field elements)
        fe opc = b0;
        opc = fe_add(fe_add(opc, opc), b1);
        opc = fe_add(fe_add(opc, opc), b2);
        opc = fe_add(fe_add(opc, opc), b3);
        opc = fe_add(fe_add(opc, opc), b4);
        // is_push = b0 (1-b1)(1-b2)(1-b3)(1-b4)  (flags.rs)
        const fe push_term = fe_mul(s0n, fe_mul(fe_mul(fe_mul(fe_mul(b0, fe_sub(one, b1)), fe_sub(one, b2)),
                                                            fe_sub(one, b3)), fe_sub(one, b4)));
        ZK_SEQ(cb, push_term.lo);
        const fe *per = periodic + (i & 127) * 9;
        fe x[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const fe c = CUR(7 + k);
            if (k < 2) stash[6 + k][tid] = c;
            x[k] = cube(c);
        }
        fe m0[4];
#pragma unroll
        for (int r2 = 0; r2 < 4; r2++) m0[r2] = fe_add(mds_row(r2, x), per[1 + r2]);
        m0[0] = fe_add(m0[0], opc);
        m0[1] = fe_add(m0[1], push_term);
        ZK_SEQ(cb, m0[3].lo);
        const fe h0 = CUR(6);
        const fe fh = fe_mul(per[0], h0);
        const fe nfh = fe_sub(h0, fh);  // (1 - hash_flag) * h0
        fe y[4];
#pragma unroll
        for (int k = 0; k < 4; k++) y[k] = fe_sub(NXT(7 + k), per[5 + k]);
        // 12..15 share the factor fh and 16..19 the factor nfh: sum the coefficient-weighted values first,
        // multiply by the flag once (ct_k (v_k f) summed = f (sum ct_k v_k): 6 multiplies fewer per row)
        fe sR = fe_zero(), sR2 = fe_zero();
        {
            // ct_r ((INV_MDS y)_r^3 - m0_r) = ct3_r (adj_r y)^3 + (-ct_r) m0_r, summed lazily
            acc288 aR = acc288_zero(), aR2 = acc288_zero();
#pragma unroll
            for (int r2 = 0; r2 < 4; r2++) {
                const fe v3 = cube(adj_row(r2, y));
                acc288_madd(aR, S.ct3[r2], v3);
                acc288_madd(aR, S.nct[r2], m0[r2]);
                if (KE == 2) {
                    acc288_madd(aR2, S.ct3b[r2], v3);
                    acc288_madd(aR2, S.nctb[r2], m0[r2]);
                }
            }
            sR = acc288_reduce(aR);
            if (KE == 2) sR2 = acc288_reduce(aR2);
        }
        t = fe_add(t, fe_mul(sR, fh));
        if (KE == 2) t2 = fe_add(t2, fe_mul(sR2, fh));
        ZK_SEQ(cb, t.lo);
        {
            const fe c7 = stash[6][tid], c8 = stash[7][tid];
            const fe d16 = fe_sub(NXT(7), c7), d17 = fe_sub(NXT(8), c8), n9 = NXT(9), n10 = NXT(10);
            acc288 aC = acc288_zero();
            acc288_madd(aC, S.ct[16], d16);
            acc288_madd(aC, S.ct[17], d17);
            acc288_madd(aC, S.ct[18], n9);
            acc288_madd(aC, S.ct[19], n10);
            t = fe_add(t, fe_mul(acc288_reduce(aC), nfh));
            if (KE == 2) {
                acc288 aD = acc288_zero();
                acc288_madd(aD, S.ct2[16], d16);
                acc288_madd(aD, S.ct2[17], d17);
                acc288_madd(aD, S.ct2[18], n9);
                acc288_madd(aD, S.ct2[19], n10);
                t2 = fe_add(t2, fe_mul(acc288_reduce(aD), nfh));
            }
        }
    }
    ZK_SEQ(cb, t.lo);
    // 0..11: degree-5 selectors (flags.rs:45-79) with shared prefixes, each consumed right away.
    // Sibling selectors share one multiply: P*(1 - b) = P - P*b.  Two pairs of constraints are folded
    // before their coefficient (3/6 and 8/9 differ only in the last bit b4):
    //   ct3*(X(1-b4))*d3 + ct6*(X b4)*d6 = X*(ct3 d3 + b4 (ct6 d6 - ct3 d3))
    //   ct8*(Z(1-b4))*d1 + ct9*(Z b4)*d1 = Z d1 * (ct8 + b4 (ct9 - ct8))
    // (exact field identities: the composition values are unchanged).
    // KE = 1: the section's terms go into one lazy 288-bit sum (one reduction instead of one per term)
    {
        constexpr bool LZ = KE == 1 && ZK_EVAL_LAZY;
        acc288 aS = acc288_zero();
#define ZK_ACCS(k, val)                                  \
    do {                                                 \
        if (LZ) acc288_madd(aS, S.ct[k], (val));    \
        else ZK_ACC(k, val);                             \
    } while (0)
#define ZK_SEQS() ZK_SEQ(cb, LZ ? aS.w[0] : (uint32_t)t.lo)
        const fe b0 = stash[0][tid], b1 = stash[1][tid], b2 = stash[2][tid], b3 = stash[3][tid], b4 = stash[4][tid];
        const fe nb0 = fe_sub(one, b0), nb2 = fe_sub(one, b2), nb3 = fe_sub(one, b3), nb4 = fe_sub(one, b4);
        const fe s0 = CUR(12), s1 = CUR(13);
        const fe s0n = stash[5][tid];  // (shadows the first section's: no live range across)
        // 0 clock, 2 shift
        ZK_ACCS(0, fe_sub(NXT(0), fe_add(CUR(0), one)));
        const fe b01 = fe_mul(b0, b1);
        ZK_ACCS(2, b01);
        const fe b0n1 = fe_sub(b0, b01);   // b0 (1-b1)
        const fe n0_1 = fe_sub(b1, b01);   // (1-b0) b1
        const fe n01 = fe_sub(nb0, n0_1);  // (1-b0)(1-b1)
        // 11 noop
        {
            const fe is_noop = fe_mul(fe_mul(fe_mul(n01, nb2), nb3), nb4);
            ZK_ACCS(11, fe_mul(is_noop, fe_sub(s0n, s0)));
        }
        ZK_SEQS();
        const fe n0_1_b2 = fe_mul(n0_1, b2);
        const fe n0_1_n2 = fe_sub(n0_1, n0_1_b2);
        const fe Y = fe_mul(n0_1_n2, b3);  // (1-b0) b1 (1-b2) b3
        fe is_add2, is_read2;
        {
            // 3 add, 6 mul: X = (1-b0) b1 (1-b2)(1-b3)
            const fe X = fe_sub(n0_1_n2, Y);
            const fe e3 = fe_mul(S.ct[3], fe_sub(s0n, fe_add(s0, s1)));
            const fe e6 = fe_mul(S.ct[6], fe_sub(s0n, fe_mul(s0, s1)));
            const fe i36 = fe_add(e3, fe_mul(b4, fe_sub(e6, e3)));
            if (LZ) acc288_madd(aS, X, i36);
            else t = fe_add(t, fe_mul(X, i36));
            if (KE == 2) {
                const fe f3 = fe_mul(S.ct2[3], fe_sub(s0n, fe_add(s0, s1)));
                const fe f6 = fe_mul(S.ct2[6], fe_sub(s0n, fe_mul(s0, s1)));
                t2 = fe_add(t2, fe_mul(X, fe_add(f3, fe_mul(b4, fe_sub(f6, f3)))));
                asm volatile("" : "+v"(t2.lo), "+v"(t2.hi));
            }
        }
        ZK_SEQS();
        {
            // 4 sadd / 5 add2 / 7 smul over the lwe_size ciphertext limbs (fhe/src/server_key.rs:89-124)
            is_add2 = fe_mul(Y, b4);
            const fe is_sadd = fe_sub(Y, is_add2);
            const fe is_smul = fe_mul(fe_mul(n0_1_b2, nb3), nb4);
            // Three column sums carry all three constraints (exact regrouping of the per-limb terms):
            //   4: sum_k (sn_k - s1_k) - delta s0           = sum_sn - sum_s1 - delta s0
            //   5: sum_k (sn_k - s_k - s_(L+k))             = sum_sn - sum_s1 - s0 - sum_hi
            //      (s_0..s_(L-1) and s_(L)..s_(2L-1) overlap s_1..s_L in all but s0 and s_(L+1)..s_(2L-1))
            //   7: sum_k (sn_k - s1_k * s0)                 = sum_sn - s0 * sum_s1
            fe sum_sn = fe_zero(), sum_s1 = fe_zero(), sum_hi = fe_zero();
            for (int k = 0; k < L; k++) {
                sum_sn = fe_add(sum_sn, NXT(12 + k));
                sum_s1 = fe_add(sum_s1, CUR(13 + k));
            }
            for (int k = 1; k < L; k++) sum_hi = fe_add(sum_hi, CUR(12 + L + k));
            const fe base = fe_sub(sum_sn, sum_s1);
            const fe acc7 = fe_sub(sum_sn, fe_mul(sum_s1, s0));
            const fe acc4 = fe_sub(base, fe_mul(S.delta, s0));  // encrypt_trivial body delta * s0 in limb L-1
            const fe acc5 = fe_sub(base, fe_add(s0, sum_hi));
            ZK_ACCS(4, fe_mul(is_sadd, acc4));
            ZK_ACCS(5, fe_mul(is_add2, acc5));
            ZK_ACCS(7, fe_mul(is_smul, acc7));
        }
        ZK_SEQS();
        {
            // 8 push / 9 read / 10 read2
            const fe p0 = fe_mul(b0n1, nb2);     // b0 (1-b1)(1-b2)
            const fe p0b3 = fe_mul(p0, b3);
            const fe p0n3 = fe_sub(p0, p0b3);
            is_read2 = fe_mul(p0b3, nb4);
            const fe zd1 = fe_mul(p0n3, fe_sub(NXT(13), s0));
            const fe i89 = fe_add(S.ct[8], fe_mul(b4, fe_sub(S.ct[9], S.ct[8])));
            if (LZ) acc288_madd(aS, zd1, i89);
            else t = fe_add(t, fe_mul(zd1, i89));
            if (KE == 2) {
                t2 = fe_add(t2, fe_mul(zd1, fe_add(S.ct2[8], fe_mul(b4, fe_sub(S.ct2[9], S.ct2[8])))));
                asm volatile("" : "+v"(t2.lo), "+v"(t2.hi));
            }
            ZK_ACCS(10, fe_mul(is_read2, fe_sub(NXT(17), s0)));
        }
        // 1 depth: (d' - d - shr + shl) - 4 read2 + 4 add2   (x4 as two doublings)
        {
            fe v = fe_add(fe_sub(fe_sub(NXT(11), CUR(11)), b0), b1);
            fe d = fe_sub(is_add2, is_read2);
            d = fe_add(d, d);
            d = fe_add(d, d);
            ZK_ACCS(1, fe_add(v, d));
        }
        if (LZ) t = fe_add(t, acc288_reduce(aS));
#undef ZK_ACCS
#undef ZK_SEQS
    }
    ZK_SEQ(cb, t.lo);
    // divisors (per-row factors from divisor_tables): transition (x^n - 1)/((x - g^(n-2))(x - g^(n-1)));
    // boundary groups (x - 1) and (x - g^(n-2)).  res = t dT + bs0 d0 + bs1 d1 as one lazy sum.
    const size_t P = map.dplane ? map.dplane : CE;
    const fe dT = divs[t_id];
    if constexpr (!BND) {
        comp[t_id] = fe_mul(t, dT);  // coset-major, like the divisor tables
        if (KE == 2) comp[plane + t_id] = fe_mul(t2, dT);
    } else {
        const fe d0 = divs[P + t_id], d1 = divs[2 * P + t_id];
        // assertions (air/src/lib.rs:170-195), sorted: step 0 -> cols 0,7,8,11,12..19 (value 0);
        // step n-2 -> cols 7,8 (program hash), 12..19 (outputs)
        acc288 a0 = acc288_zero(), a1 = acc288_zero();
        acc288_madd(a0, S.cb[0], CUR(0));
        acc288_madd(a0, S.cb[1], CUR(7));
        acc288_madd(a0, S.cb[2], CUR(8));
        acc288_madd(a0, S.cb[3], CUR(11));
        acc288_madd(a1, S.cb[12], CUR(7));
        acc288_madd(a1, S.cb[13], CUR(8));
#pragma unroll
        for (int k = 0; k < 8; k++) {
            fe c = CUR(12 + k);
            acc288_madd(a0, S.cb[4 + k], c);
            acc288_madd(a1, S.cb[14 + k], c);
        }
        // sum_k cb[12+k] (c_k - v_k) = sum_k cb[12+k] c_k - bnd1 (bnd1 precomputed on the host)
        const fe bs0 = acc288_reduce(a0), bs1 = fe_sub(acc288_reduce(a1), S.bnd1);
        acc288 aR = acc288_zero();
        acc288_madd(aR, t, dT);
        acc288_madd(aR, bs0, d0);
        acc288_madd(aR, bs1, d1);
        const fe res = acc288_reduce(aR);
        comp[t_id] = res;
        if (KE == 2) {
            ZK_SEQ(cb, res.lo);
            acc288 c0 = acc288_zero(), c1 = acc288_zero();
            acc288_madd(c0, S.cb2[0], CUR(0));
            acc288_madd(c0, S.cb2[1], CUR(7));
            acc288_madd(c0, S.cb2[2], CUR(8));
            acc288_madd(c0, S.cb2[3], CUR(11));
            acc288_madd(c1, S.cb2[12], CUR(7));
            acc288_madd(c1, S.cb2[13], CUR(8));
#pragma unroll
            for (int k = 0; k < 8; k++) {
                fe c = CUR(12 + k);
                acc288_madd(c0, S.cb2[4 + k], c);
                acc288_madd(c1, S.cb2[14 + k], c);
            }
            const fe bs0b = acc288_reduce(c0), bs1b = fe_sub(acc288_reduce(c1), S.bnd1b);
            acc288 aR2 = acc288_zero();
            acc288_madd(aR2, t2, dT);
            acc288_madd(aR2, bs0b, d0);
            acc288_madd(aR2, bs1b, d1);
            comp[plane + t_id] = acc288_reduce(aR2);
        }
    }
#undef ZK_ACC
#undef CUR
#undef NXT
}

// __constant__ memory is per device: track the upload per device (a process may run provers on
// several GPUs, and the loopback sharded prover's ranks may sit on different devices).
static std::mutex g_consts_mu;
static std::bitset<256> g_consts_done;
hipError_t upload_rescue_consts(hipStream_t st) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 256) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(g_consts_mu);
    if (g_consts_done.test((size_t)dev)) return hipSuccess;
    fe m[16];
    for (int i = 0; i < 16; i++) m[i] = fe_make(ZK_MDS[i][0], ZK_MDS[i][1]);
    e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_mds), m, sizeof m, 0, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) g_consts_done.set((size_t)dev);
    return e;
}

hipError_t eval_constraints(hipStream_t st, const fe *lde, int log_n, int log_b, const fe *periodic, const fe *divs,
                      const AirConsts *consts_dev, fe *comp, bool bnd, int nce) {
    // (with bnd the kernel reads the boundary divisor planes at stride nce * n: all 8 cosets then)
    if (bnd) nce = 8;
    return eval_constraints_mapped(st, lde, log_n, EvalMap{nce, 0, 1, log_b - 3, 1 << log_b}, periodic, divs, consts_dev, comp,
                            bnd);
}

hipError_t eval_constraints_mapped(hipStream_t st, const fe *lde, int log_n, EvalMap map, const fe *periodic,
                             const fe *divs, const AirConsts *consts_dev, fe *comp, bool bnd) {
    // the __constant__ MDS tables of this device (normally uploaded by zk_prover_create already)
    if (const hipError_t e = upload_rescue_consts(st)) return e;
    const size_t CE = (size_t)map.nce << log_n;
    const double bytes = (448.0 * (map.lshift == 0 ? 1 : 2) + (bnd ? 64.0 : 32.0)) * CE;
    if (bnd)
        ZK_PROF(st, "eval_constraints", bytes, hipLaunchKernelGGL((k_eval_constraints<1, true>), dim3(cdiv(CE, 256)), dim3(256), 0, st,
                                                                  lde, log_n, map, periodic, divs, consts_dev, consts_dev, (size_t)0, comp));
    else
        ZK_PROF(st, "eval_constraints", bytes, hipLaunchKernelGGL((k_eval_constraints<1, false>), dim3(cdiv(CE, 256)), dim3(256), 0, st,
                                                                  lde, log_n, map, periodic, divs, consts_dev, consts_dev, (size_t)0, comp));
    return hipGetLastError();
}

hipError_t eval_constraints_ext_mapped(hipStream_t st, const fe *lde, int log_n, EvalMap map, const fe *periodic,
                                 const fe *divs, const AirConsts *consts2_dev, size_t plane, fe *comp, bool bnd) {
    // the __constant__ MDS tables of this device (normally uploaded by zk_prover_create already)
    if (const hipError_t e = upload_rescue_consts(st)) return e;
    const size_t CE = (size_t)map.nce << log_n;
    const double bytes = (448.0 * (map.lshift == 0 ? 1 : 2) + (bnd ? 80.0 : 48.0)) * CE;
    if (bnd)
        ZK_PROF(st, "eval_constraints_ext", bytes, hipLaunchKernelGGL((k_eval_constraints<2, true>), dim3(cdiv(CE, 256)), dim3(256), 0,
                                                                      st, lde, log_n, map, periodic, divs, consts2_dev, consts2_dev + 1, plane, comp));
    else
        ZK_PROF(st, "eval_constraints_ext", bytes, hipLaunchKernelGGL((k_eval_constraints<2, false>), dim3(cdiv(CE, 256)), dim3(256), 0,
                                                                      st, lde, log_n, map, periodic, divs, consts2_dev, consts2_dev + 1, plane, comp));
    return hipGetLastError();
}

hipError_t eval_constraints_ext(hipStream_t st, const fe *lde, int log_n, int log_b, const fe *periodic, const fe *divs,
                          const AirConsts *consts2_dev, fe *comp, bool bnd, int nce) {
    if (bnd) nce = 8;
    return eval_constraints_ext_mapped(st, lde, log_n, EvalMap{nce, 0, 1, log_b - 3, 1 << log_b}, periodic, divs, consts2_dev,
                                (size_t)8 << log_n, comp, bnd);
}

// ================================================================ composition interpolation (K4)
__global__ void __launch_bounds__(256) k_comp_cross(CrossMap m, const fe *wi_lo, const fe *wi_hi,
                                                    const fe *i3_lo, const fe *i3_hi, fe scale, fe w8inv,
                                                    fe inv3n, int ncols, fe *polys, unsigned *nonzero) {
    for (size_t kl = blockIdx.x * (size_t)blockDim.x + threadIdx.x; kl < m.kcount; kl += (size_t)gridDim.x * blockDim.x) {
        const size_t k1 = m.k0 + kl;
        // d_r = c_r[k1] * w_8n^(-r k1)
        fe w = pow_split(wi_lo, wi_hi, k1);  // w_8n^-k1
        fe d[8];
        fe wr = fe_one();
#pragma unroll
        for (int r = 0; r < 8; r++) {
            if (r == 7 && m.derive7) {
                // the unevaluated coset: b_7 = 0 for a composition of degree < 7n (CrossMap::derive7)
                acc288 a7 = acc288_zero();
#pragma unroll
                for (int j = 0; j < 7; j++) acc288_madd(a7, m.k7[j], d[j]);
                d[7] = acc288_reduce(a7);
                break;
            }
            fe v = m.c[r][kl];
            d[r] = r ? fe_mul(v, wr) : v;
            wr = fe_mul(wr, w);
        }
        // b_k2 = sum_r w8^(-r k2) d_r  (size-8 DFT with w8^-1, direct form: 49 products avoided by radix-2)
        fe w2 = fe_mul(w8inv, w8inv), w3 = fe_mul(w2, w8inv);
        // radix-2 DIT on bit-reversed input
        fe e0 = d[0], e1 = d[4], e2 = d[2], e3 = d[6], e4 = d[1], e5 = d[5], e6 = d[3], e7 = d[7];
        fe t0 = fe_add(e0, e1), t1 = fe_sub(e0, e1), t2 = fe_add(e2, e3), t3 = fe_sub(e2, e3);
        fe t4 = fe_add(e4, e5), t5 = fe_sub(e4, e5), t6 = fe_add(e6, e7), t7 = fe_sub(e6, e7);
        t3 = fe_mul(t3, w2);
        t7 = fe_mul(t7, w2);
        fe u0 = fe_add(t0, t2), u2 = fe_sub(t0, t2), u1 = fe_add(t1, t3), u3 = fe_sub(t1, t3);
        fe u4 = fe_add(t4, t6), u6 = fe_sub(t4, t6), u5 = fe_add(t5, t7), u7 = fe_sub(t5, t7);
        u5 = fe_mul(u5, w8inv);
        u6 = fe_mul(u6, w2);
        u7 = fe_mul(u7, w3);
        fe bk[8] = {fe_add(u0, u4), fe_add(u1, u5), fe_add(u2, u6), fe_add(u3, u7),
                    fe_sub(u0, u4), fe_sub(u1, u5), fe_sub(u2, u6), fe_sub(u3, u7)};
        // a_(k1 + n k2) = b_k2 * scale * 3^-(k1 + n k2)
        fe s = fe_mul(scale, pow_split(i3_lo, i3_hi, k1));
        unsigned nz = 0;
#pragma unroll
        for (int k2 = 0; k2 < 8; k2++) {
            fe a = fe_mul(bk[k2], s);
            if (k2 < ncols) polys[(size_t)k2 * m.pstride + kl] = a;
            else nz |= !fe_is_zero(a);
            s = fe_mul(s, inv3n);
        }
        if (nz) atomicOr(nonzero, 1u);
    }
}

void comp_cross_coset(hipStream_t st, const fe *c, int log_n, const NttTables &T8n, const PowTable &inv3, fe scale,
                      fe w8inv, fe inv3n, int ncols, fe *polys, unsigned *nonzero_flag) {
    const size_t n = (size_t)1 << log_n;
    CrossMap m;
    for (int r = 0; r < 8; r++) m.c[r] = c + (size_t)r * n;
    m.k0 = 0;
    m.kcount = n;
    m.pstride = n;
    comp_cross_mapped(st, m, T8n, inv3, scale, w8inv, inv3n, ncols, polys, nonzero_flag);
}

void comp_cross_mapped(hipStream_t st, const CrossMap &m, const NttTables &T8n, const PowTable &inv3, fe scale,
                       fe w8inv, fe inv3n, int ncols, fe *polys, unsigned *nonzero_flag) {
    unsigned blocks = cdiv(m.kcount, 256);
    if (blocks > 65536) blocks = 65536;
    ZK_PROF(st, "comp_cross", (128.0 + 16.0 * ncols) * m.kcount, hipLaunchKernelGGL(k_comp_cross, dim3(blocks), dim3(256), 0, st, m, T8n.inv_lo,
                                                 T8n.inv_hi, inv3.lo, inv3.hi, scale, w8inv, inv3n, ncols, polys,
                                                 nonzero_flag));
}

// ================================================================ OOD evaluation
// One pass over every polynomial of the OOD frame: T_c(z), T_c(zg) for the trace columns and
// H_j(z) for the composition columns.  A wave owns the coefficient chunk [base, base + 64E):
// lane l sums c[base + l + 64e] * y^e (Horner in y = x^64, coalesced loads), scales by
// x^(base + l) = tab_lane[l] * tab_wave[w] and the wave reduces by shuffles.  blockIdx.y picks a
// group of OOD_GROUP polynomials so a proof launches ~5x the waves of one poly sweep.
constexpr int OOD_GROUP = 7;

__device__ __forceinline__ fe wave_sum(fe v) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        fe o;
        o.lo = __shfl_xor(v.lo, s, 64);
        o.hi = __shfl_xor(v.hi, s, 64);
        v = fe_add(v, o);
    }
    return v;
}

__global__ void k_ood_tables(fe z, fe zg, uint64_t chunk, int nw, fe *tab) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 128 + 2 * nw) return;
    fe x;
    uint64_t e;
    if (t < 128) {
        x = t < 64 ? z : zg;
        e = t & 63;
    } else {
        const int u = t - 128;
        x = u < nw ? z : zg;
        e = chunk * (uint64_t)(u < nw ? u : u - nw);
    }
    tab[t] = fe_exp(x, e);
}

template <int E>
__global__ void __launch_bounds__(256) k_ood_eval(const fe *tpolys, int W, const fe *cpolys, int C, size_t n,
                                                  const fe *tab, int nw, int w0, int w1, fe *partials) {
    const int gw = w0 + (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);  // waves [w0, w1) of nw
    const int lane = threadIdx.x & 63;
    const int tgroups = (W + OOD_GROUP - 1) / OOD_GROUP;
    const int g = blockIdx.y;
    const bool comp = g >= tgroups;
    const int p0 = comp ? 0 : g * OOD_GROUP;
    const int p1 = comp ? C : min(W, p0 + OOD_GROUP);
    const size_t base = (size_t)gw * 64 * E + lane;
    // a lane's E coefficients sit 64 apart: sum_e v_e (x^64)^e as a lazy dot product against the powers
    // (x^64)^e in LDS (one unreduced product per coefficient instead of a reduced Horner step)
    __shared__ fe Y[2][E];
    if (threadIdx.x < 2 * E) {
        const int which = threadIdx.x / E, e = threadIdx.x % E;
        const fe y = which ? fe_mul(tab[127], tab[65]) : fe_mul(tab[63], tab[1]);  // x^64
        Y[which][e] = fe_exp(y, (uint64_t)e);
    }
    __syncthreads();
    if (gw >= w1) return;
    const fe wz = fe_mul(tab[lane], tab[128 + gw]);
    const fe wzg = comp ? fe_zero() : fe_mul(tab[64 + lane], tab[128 + nw + gw]);
    for (int p = p0; p < p1; p++) {
        const fe *c = (comp ? cpolys : tpolys) + (size_t)p * n;
        fe v[E];
#pragma unroll
        for (int e = 0; e < E; e++) {
            const size_t k = base + 64 * (size_t)e;
            v[e] = k < n ? c[k] : fe_zero();
        }
        acc288 az = acc288_zero();
#pragma unroll
        for (int e = 0; e < E; e++) acc288_madd(az, v[e], Y[0][e]);
        const fe hz = wave_sum(fe_mul(acc288_reduce(az), wz));
        if (lane == 0) partials[(size_t)(comp ? 2 * W + p : p) * nw + gw] = hz;
        if (!comp) {
            acc288 ag = acc288_zero();
#pragma unroll
            for (int e = 0; e < E; e++) acc288_madd(ag, v[e], Y[1][e]);
            const fe hg = wave_sum(fe_mul(acc288_reduce(ag), wzg));
            if (lane == 0) partials[(size_t)(W + p) * nw + gw] = hg;
        }
    }
}

int ood_waves(size_t n) { return (int)std::max<size_t>(1, n / 1024); }

// part = (rank, G): only this rank's share of the coefficient range (waves [rank nw / G, (rank + 1) nw / G)), so that
// the G partial sums of each value add up to it (the sharded prover all-gathers them); (0, 1) = the whole range
void ood_eval(hipStream_t st, const fe *tpolys, int W, const fe *cpolys, int C, int log_n, fe z, fe zg, fe *tab,
              fe *partials, fe *out, int rank, int G) {
    const size_t n = (size_t)1 << log_n;
    const int E = n >= 1024 ? 16 : std::max<int>(1, (int)(n / 64));
    const int nw = (int)((n + 64 * E - 1) / (64 * E));
    const int w0 = (int)((int64_t)nw * rank / G), w1 = (int)((int64_t)nw * (rank + 1) / G);
    hipLaunchKernelGGL(k_ood_tables, dim3(cdiv(128 + 2 * nw, 256)), dim3(256), 0, st, z, zg, (uint64_t)64 * E, nw, tab);
    const dim3 grid(std::max(1u, cdiv(w1 - w0, 4)), (W + OOD_GROUP - 1) / OOD_GROUP + 1);
#define ZK_OOD(EE) hipLaunchKernelGGL((k_ood_eval<EE>), grid, dim3(256), 0, st, tpolys, W, cpolys, C, n, tab, nw, w0, w1, partials)
    const double bytes = 16.0 * (W + C) * (double)n * (w1 - w0) / nw;
    switch (E) {
        case 16: ZK_PROF(st, "ood_eval", bytes, ZK_OOD(16)); break;
        case 8: ZK_PROF(st, "ood_eval", bytes, ZK_OOD(8)); break;
        case 4: ZK_PROF(st, "ood_eval", bytes, ZK_OOD(4)); break;
        case 2: ZK_PROF(st, "ood_eval", bytes, ZK_OOD(2)); break;
        default: ZK_PROF(st, "ood_eval", bytes, ZK_OOD(1)); break;
    }
#undef ZK_OOD
    sum_partials(st, partials, 2 * W + C, nw, out, w0, w1);
}

__global__ void k_sum_partials(const fe *partials, int nblk, int b0, int b1, fe *out) {
    __shared__ fe red[256];
    fe acc = fe_zero();
    for (int b = b0 + (int)threadIdx.x; b < b1; b += blockDim.x) acc = fe_add(acc, partials[(size_t)blockIdx.x * nblk + b]);
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] = fe_add(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

void sum_partials(hipStream_t st, const fe *partials, int npolys, int nblk, fe *out, int b0, int b1) {
    if (b1 < 0) b1 = nblk;
    hipLaunchKernelGGL(k_sum_partials, dim3(npolys), dim3(256), 0, st, partials, nblk, b0, b1, out);
}

// ================================================================ DEEP composition (K6)
// ---- DEEP through coefficient form.  The trace coefficients alpha are shared by the z and zg terms
// and gamma weighs the composition columns, so with A = sum alpha_i T_i and S = A + sum gamma_j H_j
// (k1 = S(z), k2 = A(zg) exactly, since the OOD values are evaluations of the same polynomials):
//   DEEP(x) = (S(x) - S(z)) / (x - z) + (A(x) - A(zg)) / (x - zg)
// is a polynomial of degree n - 2, and (F(x) - F(c)) / (x - c) has coefficients
//   q_k = sum_{m > k} f_m c^(m-k-1) = c^-(k+1) * sum_{m > k} f_m c^m      (a suffix sum).
// So: g1_m = S_m z^m, g2_m = A_m zg^m (one pass over the 28 + 7 coefficient columns), suffix sums
// (block totals, one scan of the totals, local scans), D_k = z^-(k+1) suf1_k + zg^-(k+1) suf2_k, and one
// B-coset LDE of D gives the DEEP values: the same field values as the point-wise quotient of the 35
// LDE columns, without reading those columns (3.7 GB at 2^20) or inverting 8n denominators.
constexpr int DIV_T = 256, DIV_E = 8, DIV_CH = DIV_T * DIV_E;
static_assert(DIV_CH == ZK_DEEP_RANGE_QUANTUM, "a sharded DEEP range is whole phase-3 chunks");

// base^e for e < 2048 (lo) and base^(2048 u) for u < H (hi), 4 bases: z, zg, 1/z, 1/zg
struct DeepPowBases {
    fe b[4];
};
__global__ void k_deep_pow_tables(DeepPowBases pb, size_t H, fe *out) {
    const size_t per = 2048 + H;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= 4 * per) return;
    const size_t b = t / per, e = t % per;
    const uint64_t ex = e < 2048 ? e : 2048 * (uint64_t)(e - 2048);
    out[t] = fe_exp(pb.b[b], ex, 0);
}

__device__ __forceinline__ fe block_sum256(fe v, fe *red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    fe r = red[0];
    for (int i = 1; i < DIV_T / 64; i++) r = fe_add(r, red[i]);
    __syncthreads();
    return r;
}

// phase 1: g1, g2 and per-256 totals (one coefficient per thread)
// [kbase, kend): the coefficient range of this launch (a sharded rank's share; 0, n otherwise); n is the column stride
__global__ void __launch_bounds__(DIV_T) k_deep_div_g(const fe *tpolys, const fe *cpolys, int ccols, size_t n,
                                                     const DeepConsts *D, const fe *pw, size_t H, fe *g1, fe *g2,
                                                     fe *bs, size_t kbase, size_t kend) {
    __shared__ fe red[DIV_T / 64];
    const size_t per = 2048 + H;
    const size_t k = kbase + blockIdx.x * (size_t)DIV_T + threadIdx.x;
    fe v1 = fe_zero(), v2 = fe_zero();
    if (k < kend) {
        acc288 aA = acc288_zero(), aH = acc288_zero();
#pragma unroll 4
        for (int c = 0; c < 28; c++) acc288_madd(aA, D->alpha_t[c], ld_fe(tpolys + (size_t)c * n + k));
        for (int j = 0; j < ccols; j++) acc288_madd(aH, D->alpha_c[j], ld_fe(cpolys + (size_t)j * n + k));
        const fe A = acc288_reduce(aA);
        const fe S = fe_add(A, acc288_reduce(aH));
        v1 = fe_mul(S, pow_split(pw, pw + 2048, k));
        v2 = fe_mul(A, pow_split(pw + per, pw + per + 2048, k));
        g1[k] = v1;
        g2[k] = v2;
    }
    v1 = block_sum256(v1, red);
    v2 = block_sum256(v2, red);
    if (threadIdx.x == 0) {
        bs[2 * blockIdx.x] = v1;
        bs[2 * blockIdx.x + 1] = v2;
    }
}

// phase 2 (one block): carry[j] = sum of the totals of blocks after j (exclusive suffix), NC components
// per block entry (2: the two sums over F; 4: the two sums over E)
// total (optional): the NC sums over all nb entries (a sharded rank's range totals, exchanged between ranks)
template <int NC>
__global__ void __launch_bounds__(1024) k_deep_div_scan(fe *bs, int nb, fe *total) {
    __shared__ fe t[NC][1024];
    const int per = (nb + 1023) / 1024, lo = threadIdx.x * per, hi = min(lo + per, nb);
    fe a[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) a[c] = fe_zero();
    for (int j = lo; j < hi; j++)
#pragma unroll
        for (int c = 0; c < NC; c++) a[c] = fe_add(a[c], bs[NC * j + c]);
#pragma unroll
    for (int c = 0; c < NC; c++) t[c][threadIdx.x] = a[c];
    __syncthreads();
    // inclusive suffix scan over the 1024 thread totals (Hillis-Steele)
    for (int d = 1; d < 1024; d <<= 1) {
        fe x[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) {
            x[c] = t[c][threadIdx.x];
            if (threadIdx.x + d < 1024) x[c] = fe_add(x[c], t[c][threadIdx.x + d]);
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < NC; c++) t[c][threadIdx.x] = x[c];
        __syncthreads();
    }
    if (total && threadIdx.x == 0)
#pragma unroll
        for (int c = 0; c < NC; c++) total[c] = t[c][0];
#pragma unroll
    for (int c = 0; c < NC; c++) a[c] = threadIdx.x + 1 < 1024 ? t[c][threadIdx.x + 1] : fe_zero();
    for (int j = hi - 1; j >= lo; j--)  // exclusive suffix within this thread's entries
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const fe x = bs[NC * j + c];
            bs[NC * j + c] = a[c];
            a[c] = fe_add(a[c], x);
        }
}

// phase 3: thread owns 8 consecutive coefficients; D_k = z^-(k+1) suf1_k + zg^-(k+1) suf2_k.
// ADD: D_k is added into Dk[k] (the boundary quotient into composition column 0).  rem_flag (optional):
// set when sum_m g1_m or sum_m g2_m -- the remainders F1(z), F2(zg) of the divisions -- is nonzero.
// [kbase, n): the coefficient range (a sharded rank's share ends at n = its range end); ext (optional): the sums
// of g1, g2 over every coefficient past the range (the later ranks' totals)
template <bool ADD>
__global__ void __launch_bounds__(DIV_T) k_deep_div_q(const fe *g1, const fe *g2, const fe *carry, int nb1, size_t n,
                                                     fe z, fe zg, const fe *pw, size_t H, fe *Dk, unsigned *rem_flag,
                                                     size_t kbase, const fe *ext) {
    __shared__ fe t1[DIV_T], t2[DIV_T];
    const size_t per = 2048 + H;
    const fe *ilo = pw + 2 * per, *ihi = ilo + 2048, *jlo = pw + 3 * per, *jhi = jlo + 2048;
    const size_t k0 = kbase + blockIdx.x * (size_t)DIV_CH + (size_t)threadIdx.x * DIV_E;
    fe a[DIV_E], b[DIV_E];
    fe s1 = fe_zero(), s2 = fe_zero();
#pragma unroll
    for (int e = 0; e < DIV_E; e++) {
        const size_t k = k0 + e;
        a[e] = k < n ? ld_fe(g1 + k) : fe_zero();
        b[e] = k < n ? ld_fe(g2 + k) : fe_zero();
        s1 = fe_add(s1, a[e]);
        s2 = fe_add(s2, b[e]);
    }
    t1[threadIdx.x] = s1;
    t2[threadIdx.x] = s2;
    __syncthreads();
    for (int d = 1; d < DIV_T; d <<= 1) {
        fe x = t1[threadIdx.x], y = t2[threadIdx.x];
        if (threadIdx.x + d < DIV_T) {
            x = fe_add(x, t1[threadIdx.x + d]);
            y = fe_add(y, t2[threadIdx.x + d]);
        }
        __syncthreads();
        t1[threadIdx.x] = x;
        t2[threadIdx.x] = y;
        __syncthreads();
    }
    // R = sum of g over m >= k0 + 8: later threads of this chunk + the phase-1 blocks after it
    const int cb = min((int)blockIdx.x * (DIV_CH / DIV_T) + DIV_CH / DIV_T - 1, nb1 - 1);
    fe r1 = fe_add(carry[2 * cb], threadIdx.x + 1 < DIV_T ? t1[threadIdx.x + 1] : fe_zero());
    fe r2 = fe_add(carry[2 * cb + 1], threadIdx.x + 1 < DIV_T ? t2[threadIdx.x + 1] : fe_zero());
    if (ext) {
        r1 = fe_add(r1, ext[0]);
        r2 = fe_add(r2, ext[1]);
    }
    fe pz = pow_split(ilo, ihi, k0 + DIV_E), pg = pow_split(jlo, jhi, k0 + DIV_E);  // z^-(k+1) at k = k0 + 7
#pragma unroll
    for (int e = DIV_E - 1; e >= 0; e--) {
        const size_t k = k0 + e;
        if (k < n) {
            const fe q = fe_add(fe_mul(pz, r1), fe_mul(pg, r2));
            Dk[k] = ADD ? fe_add(ld_fe(Dk + k), q) : q;
        }
        r1 = fe_add(r1, a[e]);
        r2 = fe_add(r2, b[e]);
        pz = fe_mul(pz, z);
        pg = fe_mul(pg, zg);
    }
    if (rem_flag && k0 == 0 && !(fe_is_zero(r1) && fe_is_zero(r2))) atomicOr(rem_flag, 1u);
}

// coset-major LDE -> natural order
__global__ void __launch_bounds__(256) k_coset_to_natural(const fe *src, int log_n, int log_b, fe *out) {
    const size_t n = (size_t)1 << log_n, B = (size_t)1 << log_b, N = n << log_b;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < N; i += (size_t)gridDim.x * blockDim.x)
        out[i] = ld_fe(src + (i & (B - 1)) * n + (i >> log_b));
}

// LDE of one n-coefficient polynomial over `count` cosets r0 + stride*j: out[j*n ..] (coset-major)
void lde_cosets(hipStream_t st, const NttTables &Tn, const CosetTables &CT, const fe *coeffs, size_t n, size_t r0,
                size_t stride, int count, fe *out, fe *ntt_tmp) {
    ntt_lde(st, Tn, CT, coeffs, 0, 1, (int)r0, (int)stride, count, out, 0, n, ntt_tmp);
}

// Scratch layout (deep_poly_scratch): pw (4 power tables) | g1 (n) | g2 (n) | Dk (n) | block sums.
// A range [k0, k0 + kn) of a sharded rank (deep_range_*): the same buffers indexed by global coefficient; the range
// totals go to the block-sum area's tail (deep_range_total).
static void deep_tables(hipStream_t st, size_t n, fe z, fe zg, fe *pw) {
    const size_t H = n / 2048 + 2;  // hi[] covers every t < nb * 2048 + 8
    DeepPowBases pb;
    pb.b[0] = z;
    pb.b[1] = zg;
    pb.b[2] = fe_inv(z);
    pb.b[3] = fe_inv(zg);
    hipLaunchKernelGGL(k_deep_pow_tables, dim3(cdiv(4 * (2048 + H), 256)), dim3(256), 0, st, pb, H, pw);
}
static void deep_phase1(hipStream_t st, const fe *tpolys, const fe *cpolys, int ccols, size_t n, const DeepConsts *D,
                        fe *scratch, size_t k0, size_t kn, fe *total) {
    const size_t H = n / 2048 + 2, nb1 = (kn + DIV_T - 1) / DIV_T;
    fe *pw = scratch, *g1 = pw + 4 * (2048 + H), *g2 = g1 + n, *bs = g2 + 2 * n;
    ZK_PROF(st, "deep_combine", (16.0 * (28 + ccols) + 32.0) * kn,
            hipLaunchKernelGGL(k_deep_div_g, dim3((unsigned)nb1), dim3(DIV_T), 0, st, tpolys, cpolys, ccols, n, D, pw, H,
                               g1, g2, bs, k0, k0 + kn));
    hipLaunchKernelGGL(k_deep_div_scan<2>, dim3(1), dim3(1024), 0, st, bs, (int)nb1, total);
}
static void deep_phase3(hipStream_t st, size_t n, fe z, fe zg, fe *scratch, size_t k0, size_t kn, const fe *ext) {
    const size_t H = n / 2048 + 2, nb = (kn + DIV_CH - 1) / DIV_CH, nb1 = (kn + DIV_T - 1) / DIV_T;
    fe *pw = scratch, *g1 = pw + 4 * (2048 + H), *g2 = g1 + n, *Dk = g2 + n, *bs = Dk + n;
    ZK_PROF(st, "deep_divide", 48.0 * kn,
            hipLaunchKernelGGL(k_deep_div_q<false>, dim3((unsigned)nb), dim3(DIV_T), 0, st, g1, g2, bs, (int)nb1, k0 + kn, z,
                               zg, pw, H, Dk, nullptr, k0, ext));
}
const fe *deep_poly(hipStream_t st, const fe *tpolys, const fe *cpolys, int ccols, int log_n,
                    const void *deep_consts_dev, fe z, fe zg, fe *scratch) {
    const size_t n = (size_t)1 << log_n, H = n / 2048 + 2;
    deep_tables(st, n, z, zg, scratch);
    deep_phase1(st, tpolys, cpolys, ccols, n, (const DeepConsts *)deep_consts_dev, scratch, 0, n, nullptr);
    deep_phase3(st, n, z, zg, scratch, 0, n, nullptr);
    return scratch + 4 * (2048 + H) + 2 * n;
}
static fe *deep_range_total(fe *scratch, size_t n, int nc) {
    const size_t H = n / 2048 + 2;
    return scratch + 4 * (2048 + H) + 3 * n + (size_t)nc * ((n + DIV_T - 1) / DIV_T);
}
const fe *deep_range_begin(hipStream_t st, const fe *tpolys, const fe *cpolys, int ccols, int log_n,
                           const void *deep_consts_dev, fe z, fe zg, fe *scratch, size_t k0, size_t kn) {
    const size_t n = (size_t)1 << log_n;
    deep_tables(st, n, z, zg, scratch);
    fe *total = deep_range_total(scratch, n, 2);
    deep_phase1(st, tpolys, cpolys, ccols, n, (const DeepConsts *)deep_consts_dev, scratch, k0, kn, total);
    return total;
}
const fe *deep_range_end(hipStream_t st, int log_n, fe z, fe zg, fe *scratch, size_t k0, size_t kn, const fe *ext) {
    const size_t n = (size_t)1 << log_n, H = n / 2048 + 2;
    deep_phase3(st, n, z, zg, scratch, k0, kn, ext);
    return scratch + 4 * (2048 + H) + 2 * n;
}

// ---- boundary terms in coefficient form.  The assertion part of the composition,
//   sum_k cb_k T_ck(x) / (x - 1)  +  sum_k cb'_k (T_c'k(x) - v_k) / (x - g^(n-2)),
// is, for a trace that satisfies the assertions, a polynomial of degree n - 2: the same suffix-sum
// division as DEEP (z = 1, zg = g^(n-2)) over f0 = sum cb_k T_ck and f1 = sum cb'_k T_c'k - bnd1, added into
// composition column 0 after the interpolation.  The evaluator then skips the 22 products per CE row
// (k_eval_constraints<KE, false>); the composition coefficients are the same field values.  Nonzero
// remainders (an assertion that fails) set the degree flag.
struct BndPoly {
    fe cb[22];  // one coefficient plane (air/src/lib.rs:170-195 order: step 0 cols 0,7,8,11,12..19; step n-2 cols 7,8,12..19)
    fe bnd1;    // sum_k cb[12+k] v_k
};
// [kbase, kend): the coefficient range of this launch (a sharded rank's share; 0, n otherwise); n is the column stride
__global__ void __launch_bounds__(DIV_T) k_bnd_div_g(const fe *tpolys, size_t n, BndPoly bp, const fe *pw, size_t H,
                                                    fe *g1, fe *g2, fe *bs, size_t kbase, size_t kend) {
    __shared__ fe red[DIV_T / 64];
    const size_t per = 2048 + H;
    const size_t k = kbase + blockIdx.x * (size_t)DIV_T + threadIdx.x;
    fe v1 = fe_zero(), v2 = fe_zero();
    if (k < kend) {
        auto T = [&](int c) { return ld_fe(tpolys + (size_t)c * n + k); };
        acc288 a0 = acc288_zero(), a1 = acc288_zero();
        acc288_madd(a0, bp.cb[0], T(0));
        acc288_madd(a0, bp.cb[3], T(11));
        const fe t7 = T(7), t8 = T(8);
        acc288_madd(a0, bp.cb[1], t7);
        acc288_madd(a0, bp.cb[2], t8);
        acc288_madd(a1, bp.cb[12], t7);
        acc288_madd(a1, bp.cb[13], t8);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const fe c = T(12 + j);
            acc288_madd(a0, bp.cb[4 + j], c);
            acc288_madd(a1, bp.cb[14 + j], c);
        }
        v1 = acc288_reduce(a0);
        fe f1 = acc288_reduce(a1);
        if (k == 0) f1 = fe_sub(f1, bp.bnd1);
        v2 = fe_mul(f1, pow_split(pw + per, pw + per + 2048, k));  // f1_m (g^(n-2))^m
        g1[k] = v1;
        g2[k] = v2;
    }
    v1 = block_sum256(v1, red);
    v2 = block_sum256(v2, red);
    if (threadIdx.x == 0) {
        bs[2 * blockIdx.x] = v1;
        bs[2 * blockIdx.x + 1] = v2;
    }
}

static void bnd_tables_phase1(hipStream_t st, const fe *tpolys, size_t n, const AirConsts &K, fe c, fe *scratch,
                              size_t k0, size_t kn, fe *total) {
    const size_t H = n / 2048 + 2, nb1 = (kn + DIV_T - 1) / DIV_T;
    fe *pw = scratch, *g1 = pw + 4 * (2048 + H), *g2 = g1 + n, *bs = g2 + 2 * n;  // layout of deep_poly's scratch
    DeepPowBases pb;
    pb.b[0] = fe_one();
    pb.b[1] = c;
    pb.b[2] = fe_one();
    pb.b[3] = fe_inv(c);
    hipLaunchKernelGGL(k_deep_pow_tables, dim3(cdiv(4 * (2048 + H), 256)), dim3(256), 0, st, pb, H, pw);
    BndPoly bp;
    memcpy(bp.cb, K.coeff_b, sizeof bp.cb);
    bp.bnd1 = K.bnd1;
    ZK_PROF(st, "boundary_poly", (16.0 * 12 + 32.0) * kn,
            hipLaunchKernelGGL(k_bnd_div_g, dim3((unsigned)nb1), dim3(DIV_T), 0, st, tpolys, n, bp, pw, H, g1, g2, bs, k0,
                               k0 + kn));
    hipLaunchKernelGGL(k_deep_div_scan<2>, dim3(1), dim3(1024), 0, st, bs, (int)nb1, total);
}
static void bnd_phase3(hipStream_t st, size_t n, fe c, fe *scratch, size_t k0, size_t kn, const fe *ext, fe *col0,
                       unsigned *flag) {
    const size_t H = n / 2048 + 2, nb = (kn + DIV_CH - 1) / DIV_CH, nb1 = (kn + DIV_T - 1) / DIV_T;
    fe *pw = scratch, *g1 = pw + 4 * (2048 + H), *g2 = g1 + n, *bs = g2 + 2 * n;
    ZK_PROF(st, "boundary_poly", 64.0 * kn,
            hipLaunchKernelGGL(k_deep_div_q<true>, dim3((unsigned)nb), dim3(DIV_T), 0, st, g1, g2, bs, (int)nb1, k0 + kn,
                               fe_one(), c, pw, H, col0, flag, k0, ext));
}

void boundary_poly_add(hipStream_t st, const fe *tpolys, int log_n, const AirConsts &K, fe c, fe *scratch, fe *col0,
                       unsigned *flag) {
    const size_t n = (size_t)1 << log_n;
    bnd_tables_phase1(st, tpolys, n, K, c, scratch, 0, n, nullptr);
    bnd_phase3(st, n, c, scratch, 0, n, nullptr, col0, flag);
}

// The same over a sharded rank's coefficient range [k0, k0 + kn): begin returns the range's two sums (device); the
// ranks exchange them and end gets ext = the sums of the later ranks' ranges.  col0 is indexed by global k.
const fe *boundary_range_begin(hipStream_t st, const fe *tpolys, int log_n, const AirConsts &K, fe c, fe *scratch,
                               size_t k0, size_t kn) {
    const size_t n = (size_t)1 << log_n;
    fe *total = deep_range_total(scratch, n, 2);
    bnd_tables_phase1(st, tpolys, n, K, c, scratch, k0, kn, total);
    return total;
}
void boundary_range_end(hipStream_t st, int log_n, fe c, fe *scratch, size_t k0, size_t kn, const fe *ext, fe *col0,
                        unsigned *flag) {
    bnd_phase3(st, (size_t)1 << log_n, c, scratch, k0, kn, ext, col0, flag);
}

void deep_coeff_launch(hipStream_t st, const NttTables &Tn, const fe *tpolys, const fe *cpolys, int ccols, int log_n,
                       int log_b, const void *deep_consts_dev, fe z, fe zg, const CosetTables &CT, fe *scratch,
                       fe *ulde, fe *ntt_tmp, fe *out) {
    const size_t n = (size_t)1 << log_n, B = (size_t)1 << log_b, N = n << log_b;
    const fe *Dk = deep_poly(st, tpolys, cpolys, ccols, log_n, deep_consts_dev, z, zg, scratch);
    lde_cosets(st, Tn, CT, Dk, n, 0, 1, (int)B, ulde, ntt_tmp);
    if (!out) return;  // FRI layer 0 is read coset-major from ulde
    unsigned pb2 = cdiv(N, 256);
    if (pb2 > 65536) pb2 = 65536;
    ZK_PROF(st, "deep", 32.0 * N, hipLaunchKernelGGL(k_coset_to_natural, dim3(pb2), dim3(256), 0, st, ulde, log_n, log_b, out));
}

// ---- the same over E (FieldExtension::Quadratic): alpha_t, alpha_c, z, zg are E values; the
// composition column c is the E polynomial P_c0 + X P_c1 (base columns 2c, 2c + 1).  D is E-valued:
// its two base planes are LDE'd separately and written planar (a plane, then b plane).
struct DeepPowBasesE {
    fe2 b[4];
};
__global__ void k_deep_pow_tables_ext(DeepPowBasesE pb, size_t H, fe2 *out) {
    const size_t per = 2048 + H;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= 4 * per) return;
    const size_t b = t / per, e = t % per;
    out[t] = fe2_exp(pb.b[b], e < 2048 ? e : 2048 * (uint64_t)(e - 2048));
}
__device__ __forceinline__ fe2 pow_split2(const fe2 *lo, const fe2 *hi, size_t t) {
    return fe2_mul(lo[t & 2047], hi[t >> 11]);
}

__global__ void __launch_bounds__(DIV_T) k_deep_div_g_ext(const fe *tpolys, const fe *cpolys, int ccols, size_t n,
                                                         const DeepConstsE *D, const fe2 *pw, size_t H, fe2 *g1,
                                                         fe2 *g2, fe *bs, size_t kbase, size_t kend) {
    __shared__ fe red[DIV_T / 64];
    const size_t per = 2048 + H;
    const size_t k = kbase + blockIdx.x * (size_t)DIV_T + threadIdx.x;
    fe2 v1 = fe2_zero(), v2 = fe2_zero();
    if (k < kend) {
        acc288 aA = acc288_zero(), aB = acc288_zero();
#pragma unroll 4
        for (int c = 0; c < 28; c++) {
            const fe v = ld_fe(tpolys + (size_t)c * n + k);
            acc288_madd(aA, D->alpha_t[c].a, v);
            acc288_madd(aB, D->alpha_t[c].b, v);
        }
        acc288 hA = acc288_zero(), hB = acc288_zero();
        for (int j = 0; j < ccols; j++) {
            const fe h0 = ld_fe(cpolys + (size_t)(2 * j) * n + k), h1 = ld_fe(cpolys + (size_t)(2 * j + 1) * n + k);
            const fe2 ac = D->alpha_c[j];
            acc288_madd(hA, ac.a, h0);  // (ac.a + ac.b X)(h0 + h1 X) = (ac.a h0 + ac.b h1) + (ac.a h1 + ac.b (h0 + h1)) X
            acc288_madd(hA, ac.b, h1);
            acc288_madd(hB, ac.a, h1);
            acc288_madd(hB, ac.b, fe_add(h0, h1));
        }
        const fe2 A = fe2{acc288_reduce(aA), acc288_reduce(aB)};
        const fe2 S = fe2_add(A, fe2{acc288_reduce(hA), acc288_reduce(hB)});
        v1 = fe2_mul(S, pow_split2(pw, pw + 2048, k));
        v2 = fe2_mul(A, pow_split2(pw + per, pw + per + 2048, k));
        g1[k] = v1;
        g2[k] = v2;
    }
    const fe s0 = block_sum256(v1.a, red), s1 = block_sum256(v1.b, red), s2 = block_sum256(v2.a, red),
             s3 = block_sum256(v2.b, red);
    if (threadIdx.x == 0) {
        bs[4 * blockIdx.x] = s0;
        bs[4 * blockIdx.x + 1] = s1;
        bs[4 * blockIdx.x + 2] = s2;
        bs[4 * blockIdx.x + 3] = s3;
    }
}

__global__ void __launch_bounds__(DIV_T) k_deep_div_q_ext(const fe2 *g1, const fe2 *g2, const fe *carry, int nb1,
                                                         size_t n, fe2 z, fe2 zg, const fe2 *pw, size_t H, fe *Da,
                                                         fe *Db, size_t kbase, const fe *ext) {
    __shared__ fe2 t1[DIV_T], t2[DIV_T];
    const size_t per = 2048 + H;
    const fe2 *ilo = pw + 2 * per, *ihi = ilo + 2048, *jlo = pw + 3 * per, *jhi = jlo + 2048;
    const size_t k0 = kbase + blockIdx.x * (size_t)DIV_CH + (size_t)threadIdx.x * DIV_E;
    fe2 s1 = fe2_zero(), s2 = fe2_zero();
    for (int e = 0; e < DIV_E; e++) {
        const size_t k = k0 + e;
        if (k < n) {
            s1 = fe2_add(s1, g1[k]);
            s2 = fe2_add(s2, g2[k]);
        }
    }
    t1[threadIdx.x] = s1;
    t2[threadIdx.x] = s2;
    __syncthreads();
    for (int d = 1; d < DIV_T; d <<= 1) {
        fe2 x = t1[threadIdx.x], y = t2[threadIdx.x];
        if (threadIdx.x + d < DIV_T) {
            x = fe2_add(x, t1[threadIdx.x + d]);
            y = fe2_add(y, t2[threadIdx.x + d]);
        }
        __syncthreads();
        t1[threadIdx.x] = x;
        t2[threadIdx.x] = y;
        __syncthreads();
    }
    const int cb = min((int)blockIdx.x * (DIV_CH / DIV_T) + DIV_CH / DIV_T - 1, nb1 - 1);
    fe2 r1 = fe2_add(fe2{carry[4 * cb], carry[4 * cb + 1]}, threadIdx.x + 1 < DIV_T ? t1[threadIdx.x + 1] : fe2_zero());
    fe2 r2 = fe2_add(fe2{carry[4 * cb + 2], carry[4 * cb + 3]}, threadIdx.x + 1 < DIV_T ? t2[threadIdx.x + 1] : fe2_zero());
    if (ext) {
        r1 = fe2_add(r1, fe2{ext[0], ext[1]});
        r2 = fe2_add(r2, fe2{ext[2], ext[3]});
    }
    fe2 pz = pow_split2(ilo, ihi, k0 + DIV_E), pg = pow_split2(jlo, jhi, k0 + DIV_E);
    for (int e = DIV_E - 1; e >= 0; e--) {
        const size_t k = k0 + e;
        if (k < n) {
            const fe2 d = fe2_add(fe2_mul(pz, r1), fe2_mul(pg, r2));
            Da[k] = d.a;
            Db[k] = d.b;
            r1 = fe2_add(r1, g1[k]);
            r2 = fe2_add(r2, g2[k]);
        }
        pz = fe2_mul(pz, z);
        pg = fe2_mul(pg, zg);
    }
}

// scratch layout (E): pw (4 E power tables) | g1 (n E) | g2 (n E) | Da (n) | Db (n) | block sums (4 per block)
static void deep_tables_ext(hipStream_t st, size_t n, fe2 z, fe2 zg, fe *scratch) {
    const size_t H = n / 2048 + 2;
    DeepPowBasesE pb;
    pb.b[0] = z;
    pb.b[1] = zg;
    pb.b[2] = fe2_inv(z);
    pb.b[3] = fe2_inv(zg);
    hipLaunchKernelGGL(k_deep_pow_tables_ext, dim3(cdiv(4 * (2048 + H), 256)), dim3(256), 0, st, pb, H, (fe2 *)scratch);
}
static void deep_phase1_ext(hipStream_t st, const fe *tpolys, const fe *cpolys, int ccols, size_t n,
                            const DeepConstsE *D, fe *scratch, size_t k0, size_t kn, fe *total) {
    const size_t H = n / 2048 + 2, nb1 = (kn + DIV_T - 1) / DIV_T;
    fe2 *pw = (fe2 *)scratch, *g1 = pw + 4 * (2048 + H), *g2 = g1 + n;
    fe *bs = (fe *)(g2 + n) + 2 * n;
    ZK_PROF(st, "deep_combine", (16.0 * (28 + 2 * ccols) + 64.0) * kn,
            hipLaunchKernelGGL(k_deep_div_g_ext, dim3((unsigned)nb1), dim3(DIV_T), 0, st, tpolys, cpolys, ccols, n, D, pw,
                               H, g1, g2, bs, k0, k0 + kn));
    hipLaunchKernelGGL(k_deep_div_scan<4>, dim3(1), dim3(1024), 0, st, bs, (int)nb1, total);
}
static void deep_phase3_ext(hipStream_t st, size_t n, fe2 z, fe2 zg, fe *scratch, size_t k0, size_t kn, const fe *ext) {
    const size_t H = n / 2048 + 2, nb = (kn + DIV_CH - 1) / DIV_CH, nb1 = (kn + DIV_T - 1) / DIV_T;
    fe2 *pw = (fe2 *)scratch, *g1 = pw + 4 * (2048 + H), *g2 = g1 + n;
    fe *Da = (fe *)(g2 + n), *Db = Da + n, *bs = Db + n;
    ZK_PROF(st, "deep_divide", 96.0 * kn,
            hipLaunchKernelGGL(k_deep_div_q_ext, dim3((unsigned)nb), dim3(DIV_T), 0, st, g1, g2, bs, (int)nb1, k0 + kn, z, zg,
                               pw, H, Da, Db, k0, ext));
}
const fe *deep_poly_ext(hipStream_t st, const fe *tpolys, const fe *cpolys, int ccols, int log_n,
                        const void *deep_consts_dev, fe2 z, fe2 zg, fe *scratch) {
    const size_t n = (size_t)1 << log_n, H = n / 2048 + 2;
    deep_tables_ext(st, n, z, zg, scratch);
    deep_phase1_ext(st, tpolys, cpolys, ccols, n, (const DeepConstsE *)deep_consts_dev, scratch, 0, n, nullptr);
    deep_phase3_ext(st, n, z, zg, scratch, 0, n, nullptr);
    return (fe *)((fe2 *)scratch + 4 * (2048 + H) + 2 * n);  // planes Da, Da + n
}
static fe *deep_range_total_ext(fe *scratch, size_t n) {
    const size_t H = n / 2048 + 2;
    return (fe *)((fe2 *)scratch + 4 * (2048 + H) + 2 * n) + 2 * n + 4 * ((n + DIV_T - 1) / DIV_T);
}
const fe *deep_range_begin_ext(hipStream_t st, const fe *tpolys, const fe *cpolys, int ccols, int log_n,
                               const void *deep_consts_dev, fe2 z, fe2 zg, fe *scratch, size_t k0, size_t kn) {
    const size_t n = (size_t)1 << log_n;
    deep_tables_ext(st, n, z, zg, scratch);
    fe *total = deep_range_total_ext(scratch, n);
    deep_phase1_ext(st, tpolys, cpolys, ccols, n, (const DeepConstsE *)deep_consts_dev, scratch, k0, kn, total);
    return total;
}
const fe *deep_range_end_ext(hipStream_t st, int log_n, fe2 z, fe2 zg, fe *scratch, size_t k0, size_t kn,
                             const fe *ext) {
    const size_t n = (size_t)1 << log_n, H = n / 2048 + 2;
    deep_phase3_ext(st, n, z, zg, scratch, k0, kn, ext);
    return (fe *)((fe2 *)scratch + 4 * (2048 + H) + 2 * n);
}

void deep_coeff_ext_launch(hipStream_t st, const NttTables &Tn, const fe *tpolys, const fe *cpolys, int ccols,
                           int log_n, int log_b, const void *deep_consts_dev, fe2 z, fe2 zg, const CosetTables &CT,
                           fe *scratch, fe *ulde, fe *ntt_tmp, fe *out) {
    const size_t n = (size_t)1 << log_n, B = (size_t)1 << log_b, N = n << log_b;
    const fe *Dk = deep_poly_ext(st, tpolys, cpolys, ccols, log_n, deep_consts_dev, z, zg, scratch);
    for (int plane = 0; plane < 2; plane++) lde_cosets(st, Tn, CT, Dk + plane * n, n, 0, 1, (int)B, ulde + plane * N, ntt_tmp);
    if (!out) return;
    unsigned pb2 = cdiv(N, 256);
    if (pb2 > 65536) pb2 = 65536;
    for (int plane = 0; plane < 2; plane++)
        ZK_PROF(st, "deep", 32.0 * N,
                hipLaunchKernelGGL(k_coset_to_natural, dim3(pb2), dim3(256), 0, st, ulde + plane * N, log_n, log_b, out + plane * N));
}

// ================================================================ FRI transcript on the device
// DefaultRandomCoin<Blake3_256> for the FRI commit phase without a host round trip per layer:
// seed = merge(seed, root) (the layer root is nodes[1]), then draw: counter = 1, 2, ...,
// merge_with_int(seed, counter) = BLAKE3(seed || counter_le64) until the first 16 bytes (k = 1) or
// both 16-byte halves (k = 2) are canonical.  alpha goes to *alpha_out (the fold kernel's constants).
// The host replays the same transcript from the downloaded roots (same alphas, checked).
__device__ __forceinline__ bool fe_canon_dev(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    const uint64_t lo = (uint64_t)w0 | ((uint64_t)w1 << 32), hi = (uint64_t)w2 | ((uint64_t)w3 << 32);
    return !(hi == ZK_P_HI && lo >= ZK_P_LO);
}
__global__ void k_fri_coin(uint32_t *seed, const uint8_t *root, int k, fe *alpha_out, fe *alpha_log) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint32_t s[8], r[8], h[8];
    for (int i = 0; i < 8; i++) s[i] = seed[i];
    load_digest(root, r);
    b3::merge(s, r, h);
    for (int i = 0; i < 8; i++) seed[i] = h[i];
    for (uint32_t ctr = 1; ctr < 1000; ctr++) {
        uint32_t m[16] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], ctr, 0, 0, 0, 0, 0, 0, 0};
        uint32_t d[8];
        b3::iv(d);
        b3::compress(d, m, 0, 0, 40, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT);
        if (fe_canon_dev(d[0], d[1], d[2], d[3]) && (k == 1 || fe_canon_dev(d[4], d[5], d[6], d[7]))) {
            const fe a0 = fe{(uint64_t)d[0] | ((uint64_t)d[1] << 32), (uint64_t)d[2] | ((uint64_t)d[3] << 32)};
            const fe a1 = fe{(uint64_t)d[4] | ((uint64_t)d[5] << 32), (uint64_t)d[6] | ((uint64_t)d[7] << 32)};
            alpha_out[0] = alpha_log[0] = a0;
            if (k == 2) alpha_out[1] = alpha_log[1] = a1;
            return;
        }
    }
}

void fri_coin_launch(hipStream_t st, uint32_t *seed_dev, const uint8_t *root_dev, int k, fe *alpha_dev,
                     fe *alpha_log) {
    hipLaunchKernelGGL(k_fri_coin, dim3(1), dim3(64), 0, st, seed_dev, root_dev, k, alpha_dev, alpha_log);
}

// ================================================================ FRI fold (K7)
// next[r] = p_r(alpha), p_r of degree < fold interpolating the layer values at x_r * zeta^k:
//   p_r(alpha) = (1/fold) * sum_m V_m (alpha / x_r)^m,  V_m = sum_k v_k zeta^(-k m)
// V_m = sum_k v_k * zeta^(-k m), m < F: idft_small (fri_small.hpp)

// One FRI fold: row r = [e(r + k*rows)] at x_r * zeta^k -> the degree-respecting projection at alpha:
// sum_m V_m (alpha / x_r)^m / F, with x_r = offset * w_L^r.
template <int F>
__global__ void __launch_bounds__(256) k_fri_fold(const fe *layer, size_t L, const FoldConsts *Fc, const fe *wi_lo,
                                                  const fe *wi_hi, size_t wstride, FriLayout f, fe *next) {
    const size_t rows = L / F;
    for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < rows; r += (size_t)gridDim.x * blockDim.x) {
        fe v[F];
#pragma unroll
        for (int k = 0; k < F; k++) v[k] = layer[fri_at(f, r + (size_t)k * rows)];
        // beta = alpha / x_r, 1/x_r = offset^-1 * w_L^-r = offset^-1 * w_N^(-r*wstride)
        const fe beta = fe_mul(Fc->alpha, fe_mul(Fc->inv_offset, pow_split(wi_lo, wi_hi, r * wstride)));
        idft_small<F>(v, Fc->zinv);
        fe acc = v[F - 1];
#pragma unroll
        for (int m = F - 2; m >= 0; m--) acc = fe_add(fe_mul(acc, beta), v[m]);
        next[r] = fe_mul(acc, Fc->inv_fold);
    }
}

void fri_fold_launch(hipStream_t st, const fe *layer, size_t L, int fold, const void *fold_consts_dev,
                     const NttTables &TN, size_t wstride, fe *next, int lb) {
    unsigned blocks = cdiv(L / fold, 256);
    if (blocks > 65536) blocks = 65536;
    const FoldConsts *F = (const FoldConsts *)fold_consts_dev;
    const FriLayout fl = fri_layout(L, lb);
#define ZK_FOLD(FF) ZK_PROF(st, "fri_fold", 16.0 * L + 16.0 * (L / fold), hipLaunchKernelGGL((k_fri_fold<FF>), dim3(blocks), dim3(256), 0, st, layer, L, F, TN.inv_lo, TN.inv_hi, wstride, fl, next))
    switch (fold) {
        case 2: ZK_FOLD(2); break;
        case 4: ZK_FOLD(4); break;
        case 8: ZK_FOLD(8); break;
        default: ZK_FOLD(16); break;
    }
#undef ZK_FOLD
}

// ================================================================ FieldExtension::Quadratic (K5-K7 over E)
// OOD over E points: the same wave layout as k_ood_eval, E-valued powers.
__global__ void k_ood_tables_ext(fe2 z, fe2 zg, uint64_t chunk, int nw, fe2 *tab) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 128 + 2 * nw) return;
    fe2 x;
    uint64_t e;
    if (t < 128) {
        x = t < 64 ? z : zg;
        e = t & 63;
    } else {
        const int u = t - 128;
        x = u < nw ? z : zg;
        e = chunk * (uint64_t)(u < nw ? u : u - nw);
    }
    tab[t] = fe2_exp(x, e);
}

// sum_e v_e y_e over E with base coefficients v: two lazy dot products (a and b components of y)
template <int E>
__device__ __forceinline__ fe2 dot_base_ext(const fe *v, const fe2 *y) {
    acc288 aa = acc288_zero(), ab = acc288_zero();
#pragma unroll
    for (int e = 0; e < E; e++) {
        const fe2 w = y[e];
        acc288_madd(aa, v[e], w.a);
        acc288_madd(ab, v[e], w.b);
    }
    return fe2{acc288_reduce(aa), acc288_reduce(ab)};
}

template <int E>
__global__ void __launch_bounds__(256) k_ood_eval_ext(const fe *tpolys, int W, const fe *cpolys, int C, size_t n,
                                                      const fe2 *tab, int nw, int w0, int w1, fe *partials) {
    const int gw = w0 + (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);  // waves [w0, w1) of nw
    const int lane = threadIdx.x & 63;
    const int np = 2 * W + C;
    const int tgroups = (W + OOD_GROUP - 1) / OOD_GROUP;
    const int g = blockIdx.y;
    const bool comp = g >= tgroups;
    const int p0 = comp ? 0 : g * OOD_GROUP;
    const int p1 = comp ? C : min(W, p0 + OOD_GROUP);
    const size_t base = (size_t)gw * 64 * E + lane;
    // powers (x^64)^e in LDS: the lane's strided sum is a base x E dot product (see k_ood_eval)
    __shared__ fe2 Y[2][E];
    if (threadIdx.x < 2 * E) {
        const int which = threadIdx.x / E, e = threadIdx.x % E;
        const fe2 y = which ? fe2_mul(tab[127], tab[65]) : fe2_mul(tab[63], tab[1]);  // x^64
        Y[which][e] = fe2_exp(y, (uint64_t)e);
    }
    __syncthreads();
    if (gw >= w1) return;
    const fe2 wz = fe2_mul(tab[lane], tab[128 + gw]);
    const fe2 wzg = comp ? fe2_zero() : fe2_mul(tab[64 + lane], tab[128 + nw + gw]);
    for (int p = p0; p < p1; p++) {
        const fe *c = (comp ? cpolys : tpolys) + (size_t)p * n;
        fe v[E];
#pragma unroll
        for (int e = 0; e < E; e++) {
            const size_t k = base + 64 * (size_t)e;
            v[e] = k < n ? c[k] : fe_zero();
        }
        const fe2 hz = fe2_mul(dot_base_ext<E>(v, Y[0]), wz);
        const fe sa = wave_sum(hz.a), sb = wave_sum(hz.b);
        const int slot = comp ? 2 * W + p : p;
        if (lane == 0) {
            partials[(size_t)slot * nw + gw] = sa;
            partials[(size_t)(np + slot) * nw + gw] = sb;
        }
        if (!comp) {
            const fe2 hg = fe2_mul(dot_base_ext<E>(v, Y[1]), wzg);
            const fe ga = wave_sum(hg.a), gb = wave_sum(hg.b);
            if (lane == 0) {
                partials[(size_t)(W + p) * nw + gw] = ga;
                partials[(size_t)(np + W + p) * nw + gw] = gb;
            }
        }
    }
}

void ood_eval_ext(hipStream_t st, const fe *tpolys, int W, const fe *cpolys, int C, int log_n, fe2 z, fe2 zg,
                  fe *tab, fe *partials, fe *out, int rank, int G) {
    const size_t n = (size_t)1 << log_n;
    const int E = n >= 1024 ? 16 : std::max<int>(1, (int)(n / 64));
    const int nw = (int)((n + 64 * E - 1) / (64 * E));
    const int w0 = (int)((int64_t)nw * rank / G), w1 = (int)((int64_t)nw * (rank + 1) / G);
    fe2 *t2 = reinterpret_cast<fe2 *>(tab);
    hipLaunchKernelGGL(k_ood_tables_ext, dim3(cdiv(128 + 2 * nw, 256)), dim3(256), 0, st, z, zg, (uint64_t)64 * E, nw, t2);
    const dim3 grid(std::max(1u, cdiv(w1 - w0, 4)), (W + OOD_GROUP - 1) / OOD_GROUP + 1);
#define ZK_OOD(EE) hipLaunchKernelGGL((k_ood_eval_ext<EE>), grid, dim3(256), 0, st, tpolys, W, cpolys, C, n, t2, nw, w0, w1, partials)
    const double bytes = 16.0 * (W + C) * (double)n * (w1 - w0) / nw;
    switch (E) {
        case 16: ZK_PROF(st, "ood_eval_ext", bytes, ZK_OOD(16)); break;
        case 8: ZK_PROF(st, "ood_eval_ext", bytes, ZK_OOD(8)); break;
        case 4: ZK_PROF(st, "ood_eval_ext", bytes, ZK_OOD(4)); break;
        case 2: ZK_PROF(st, "ood_eval_ext", bytes, ZK_OOD(2)); break;
        default: ZK_PROF(st, "ood_eval_ext", bytes, ZK_OOD(1)); break;
    }
#undef ZK_OOD
    sum_partials(st, partials, 2 * (2 * W + C), nw, out, w0, w1);
}

// 1 / (N(x - z) N(x - zg)): N(x - z) = (x - z.a)(x - z.a - z.b) - z.b^2 (the norm of x - z, X^2 = X + 1)
__device__ __forceinline__ fe norm_pair_denominator(const fe *xr, const fe *wlo, const fe *whi, size_t i, int log_n,
                                                    fe2 z, fe2 zg, fe zb2, fe zgb2) {
    const fe x = fe_mul(xr[i >> log_n], pow_split(wlo, whi, i & (((size_t)1 << log_n) - 1)));
    const fe xa = fe_sub(x, z.a), ga = fe_sub(x, zg.a);
    const fe d1 = fe_sub(fe_mul(xa, fe_sub(xa, z.b)), zb2);
    const fe d2 = fe_sub(fe_mul(ga, fe_sub(ga, zg.b)), zgb2);
    return fe_mul(d1, d2);
}

__global__ void __launch_bounds__(256) k_batch_inv_norm_pairs(const fe *xr, int log_b, int log_n, const fe *wlo,
                                                              const fe *whi, fe2 z, fe2 zg, fe zb2, fe zgb2, fe *out,
                                                              size_t total_threads) {
    const size_t N = (size_t)1 << (log_n + log_b);
    const size_t T = total_threads;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= T) return;
    fe acc = fe_one();
#pragma unroll 4
    for (int k = 0; k < INV_K; k++) {
        const size_t i = t + (size_t)k * T;
        if (i < N) {
            acc = fe_mul(acc, norm_pair_denominator(xr, wlo, whi, i, log_n, z, zg, zb2, zgb2));
            out[i] = acc;
        }
    }
    fe inv = fe_inv(acc);
#pragma unroll 4
    for (int k = INV_K - 1; k >= 0; k--) {
        const size_t i = t + (size_t)k * T;
        if (i >= N) continue;
        const fe d = norm_pair_denominator(xr, wlo, whi, i, log_n, z, zg, zb2, zgb2);
        out[i] = k > 0 ? fe_mul(inv, out[i - T]) : inv;
        inv = fe_mul(inv, d);
    }
}

void batch_inv_norm_pairs(hipStream_t st, const NttTables &Tn, const fe *xr, int log_b, int log_n, fe2 z, fe2 zg,
                          fe *out) {
    const size_t N = (size_t)1 << (log_n + log_b);
    const size_t threads = (N + INV_K - 1) / INV_K;
    const fe zb2 = fe_mul(z.b, z.b), zgb2 = fe_mul(zg.b, zg.b);
    ZK_PROF(st, "batch_inv_ext", 16.0 * N, hipLaunchKernelGGL(k_batch_inv_norm_pairs, dim3(cdiv(threads, 256)), dim3(256), 0, st, xr,
                                                    log_b, log_n, Tn.fwd_lo, Tn.fwd_hi, z, zg, zb2, zgb2, out, threads));
}

// FRI row r over E: [e(r + k rows)]_k, each value hashed as (a, b)
__global__ void __launch_bounds__(256) k_hash_fri_rows_ext(const fe *layer, size_t L, int fold, FriLayout f, uint8_t *leaves) {
    const size_t rows = L / fold;
    for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < rows; r += (size_t)gridDim.x * blockDim.x) {
        uint32_t h[8];
        b3::hash_elements(2 * fold, [&](int t) { return layer[(size_t)(t & 1) * L + fri_at(f, r + (size_t)(t >> 1) * rows)]; }, h);
        store_digest(leaves + 32 * r, h);
    }
}

void commit_fri_layer_ext(hipStream_t st, const fe *layer, size_t L, int fold, uint8_t *leaves, uint8_t *nodes, int lb) {
    const size_t rows = L / fold;
    const FriLayout f = fri_layout(L, lb);
    ZK_PROF(st, "hash_fri_rows_ext", 32.0 * L + 32.0 * rows, hipLaunchKernelGGL(k_hash_fri_rows_ext, dim3(cdiv(rows, 256)), dim3(256), 0, st, layer, L, fold, f, leaves));
    merkle_tree(st, leaves, rows, nodes);
}

// FRI fold over E: the interpolation is F-linear, so each component goes through idft_small and the
// resulting E coefficients are evaluated at beta = alpha / x_r by an E Horner.
template <int F>
__global__ void __launch_bounds__(256) k_fri_fold_ext(const fe *layer, size_t L, const FoldConstsE *Fc, const fe *wi_lo,
                                                      const fe *wi_hi, size_t wstride, FriLayout f, fe *next) {
    const size_t rows = L / F;
    for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < rows; r += (size_t)gridDim.x * blockDim.x) {
        fe va[F], vb[F];
#pragma unroll
        for (int k = 0; k < F; k++) {
            const size_t at = fri_at(f, r + (size_t)k * rows);
            va[k] = layer[at];
            vb[k] = layer[L + at];
        }
        const fe2 beta = fe2_mulb(Fc->alpha, fe_mul(Fc->inv_offset, pow_split(wi_lo, wi_hi, r * wstride)));
        idft_small<F>(va, Fc->zinv);
        idft_small<F>(vb, Fc->zinv);
        fe2 acc = fe2{va[F - 1], vb[F - 1]};
#pragma unroll
        for (int m = F - 2; m >= 0; m--) acc = fe2_add(fe2_mul(acc, beta), fe2{va[m], vb[m]});
        acc = fe2_mulb(acc, Fc->inv_fold);
        next[r] = acc.a;
        next[rows + r] = acc.b;
    }
}

void fri_fold_ext_launch(hipStream_t st, const fe *layer, size_t L, int fold, const void *fold_consts_dev,
                         const NttTables &TN, size_t wstride, fe *next, int lb) {
    unsigned blocks = cdiv(L / fold, 256);
    if (blocks > 65536) blocks = 65536;
    const FoldConstsE *F = (const FoldConstsE *)fold_consts_dev;
    const FriLayout fl = fri_layout(L, lb);
#define ZK_FOLD(FF) ZK_PROF(st, "fri_fold_ext", 32.0 * L + 32.0 * (L / fold), hipLaunchKernelGGL((k_fri_fold_ext<FF>), dim3(blocks), dim3(256), 0, st, layer, L, F, TN.inv_lo, TN.inv_hi, wstride, fl, next))
    switch (fold) {
        case 2: ZK_FOLD(2); break;
        case 4: ZK_FOLD(4); break;
        case 8: ZK_FOLD(8); break;
        default: ZK_FOLD(16); break;
    }
#undef ZK_FOLD
}

// ================================================================ elementwise helpers
__global__ void k_coset_major_to_natural(const fe *src, int log_n, int log_b, fe *dst) {
    size_t N = (size_t)1 << (log_n + log_b), n = (size_t)1 << log_n, B = (size_t)1 << log_b;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < N; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[(i & (B - 1)) * n + (i >> log_b)];
}

__global__ void k_gather_chunks(const uint64_t *addr, size_t k, fe *out) {
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t < k) out[t] = *reinterpret_cast<const fe *>((uintptr_t)addr[t]);
}

__global__ void __launch_bounds__(256) k_copy_to_host(CopyList L) {
    const int e = blockIdx.y;
    if (e >= L.n) return;
    const uint32_t *src = L.src[e];
    uint32_t *dst = L.dst[e];
    for (size_t w = blockIdx.x * (size_t)blockDim.x + threadIdx.x; w < L.words[e]; w += (size_t)gridDim.x * blockDim.x)
        dst[w] = src[w];
    __threadfence_system();
}

hipError_t copy_to_host(hipStream_t st, const CopyList &L, size_t max_words) {
    if (L.n <= 0) return hipSuccess;
    const unsigned bx = std::max(1u, std::min(cdiv(max_words, 256), 64u));
    hipLaunchKernelGGL(k_copy_to_host, dim3(bx, (unsigned)L.n), dim3(256), 0, st, L);
    return hipGetLastError();  // a failed launch must not let d2h_flush deliver stale staging bytes
}

void gather_chunks(hipStream_t st, const uint64_t *addr, size_t k, fe *out) {
    if (k) ZK_PROF(st, "gather_chunks", 24.0 * k, hipLaunchKernelGGL(k_gather_chunks, dim3(cdiv(k, 256)), dim3(256), 0, st, addr, k, out));
}

__global__ void k_gather_fe(const fe *src, const uint64_t *idx, size_t k, fe *out) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t < k) out[t] = src[idx[t]];
}

void gather_fe(hipStream_t st, const fe *src, const uint64_t *idx, size_t k, fe *out) {
    if (k) hipLaunchKernelGGL(k_gather_fe, dim3(cdiv(k, 64)), dim3(64), 0, st, src, idx, k, out);
}

KernelProfiler &profiler() {
    static KernelProfiler p;
    return p;
}

void coset_major_to_natural(hipStream_t st, const fe *src, int log_n, int log_b, fe *dst) {
    size_t N = (size_t)1 << (log_n + log_b);
    unsigned blocks = cdiv(N, 256);
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_coset_major_to_natural, dim3(blocks), dim3(256), 0, st, src, log_n, log_b, dst);
}

}  // namespace zk

// ================================================================ diagnostics (C ABI: zk_diag_*)
namespace zk {
__global__ void k_field_op(int op, const fe *a, const fe *b, fe *out, size_t count) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= count) return;
    fe x = a[t], y = b[t];
    fe r;
    switch (op) {
    case 0: r = fe_add(x, y); break;
    case 1: r = fe_sub(x, y); break;
    case 2: r = fe_mul(x, y); break;
    case 3: r = fe_inv(x); break;
    case 5: r = fe_add_lazy(x, y); break;  // the NTT's lazy forms: x any value < 2^128, y canonical
    case 6: r = fe_canon(x); break;
    case 7: r = fe_mul_w2(x, fe_w2{y, fe_mul(y, fe{0, 1})}); break;  // two-part constant (w, w 2^64)
    case 8:
    case 9:
    case 10: {
        // the NTT butterflies' addsub2 forms (V = op - 8: both sums canonical, both lazy, first lazy): inputs (x, y) and
        // (a, b)[count - 1 - t]; lane t returns output t & 3 of (x + y, x - y, x2 + y2, x2 - y2)
        const fe x2 = a[count - 1 - t], y2 = b[count - 1 - t];
        fe o[4];
        if (op == 8) addsub2_v<0>(x, y, x2, y2, o[0], o[1], o[2], o[3]);
        else if (op == 9) addsub2_v<1>(x, y, x2, y2, o[0], o[1], o[2], o[3]);
        else addsub2_v<2>(x, y, x2, y2, o[0], o[1], o[2], o[3]);
        r = o[t & 3];
        break;
    }
    default: r = fe_exp(x, y.lo, y.hi); break;
    }
    out[t] = r;
}

__global__ void k_blake3_elems(const fe *in, int k, size_t count, uint8_t *out) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= count) return;
    uint32_t h[8];
    b3::hash_elements(k, [&](int i) { return in[t * k + i]; }, h);
    store_digest(out + 32 * t, h);
}

void diag_field_op(hipStream_t st, int op, const fe *a, const fe *b, fe *out, size_t count) {
    hipLaunchKernelGGL(k_field_op, dim3(cdiv(count, 256)), dim3(256), 0, st, op, a, b, out, count);
}
void diag_blake3_elems(hipStream_t st, const fe *in, int k, size_t count, uint8_t *out) {
    hipLaunchKernelGGL(k_blake3_elems, dim3(cdiv(count, 256)), dim3(256), 0, st, in, k, count, out);
}
}  // namespace zk
