// NTT design lab: the library's four-step pass-2 kernel (ntt_pass2<10, 4096>: 1024 threads, one radix-4
// butterfly per thread per LDS round, a block barrier per round) against experimental layouts of the
// same 1024-point line transforms, on 28 x 2^20 elements.  Outputs are compared bit for bit.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../encrypt-zkvm_amd/csrc -I../../include ntt_lab.hip -o ntt_lab
#include "../../encrypt-zkvm_amd/csrc/kernels.hip"
#include "../../encrypt-zkvm_amd/csrc/host_field.hpp"
#include <stdio.h>
#include <vector>
#include "fmul_variants.hpp"

using namespace zk;

// ---------------------------------------------------------------- wave-per-line pass 2 (LOGM = 10)
// A block = 4 waves = 4 adjacent lines (64-B row segments, as in the library kernel).  Global loads and
// stores go through the LDS tile with one block barrier each; in between every wave transforms its own
// 1024-point line with 16 elements per lane in registers: 1024 = 16 x 16 x 4,
//   lane a holds x[a + 64 b] -> 16-point DFT over b -> * w1024^(a c) -> LDS exchange ->
//   lane (c, a0) holds Z[a0 + 4 a1][c] -> 16-point DFT over a1 -> * w64^(a0 d0) -> LDS exchange ->
//   lane (c, q) holds V_a0[4q + r] -> 4-point DFTs over a0 -> X[c + 16 (4q + r) + 256 d1].
// Wave-local LDS traffic needs no barrier (a wave's LDS operations complete in order).
struct W16 {
    fe w[8];  // w16^0..7
    fe w4;    // w4 = w16^4
};

__device__ __forceinline__ void bfly(fe &a, fe &b, fe w) {
    const fe t = fe_mul(b, w);
    b = fe_sub(a, t);
    a = fe_add(a, t);
}
__device__ __forceinline__ void bfly1(fe &a, fe &b) {
    const fe t = b;
    b = fe_sub(a, t);
    a = fe_add(a, t);
}

// in-register 16-point DFT, natural order in and out: y[c] = sum_b x[b] w16^(b c)
__device__ __forceinline__ void dft16(fe x[16], const W16 &W) {
    fe v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = x[((i & 1) << 3) | ((i & 2) << 1) | ((i & 4) >> 1) | ((i & 8) >> 3)];
#pragma unroll
    for (int g = 0; g < 16; g += 2) bfly1(v[g], v[g + 1]);
#pragma unroll
    for (int g = 0; g < 16; g += 4) {
        bfly1(v[g], v[g + 2]);
        bfly(v[g + 1], v[g + 3], W.w[4]);
    }
#pragma unroll
    for (int g = 0; g < 16; g += 8) {
        bfly1(v[g], v[g + 4]);
#pragma unroll
        for (int j = 1; j < 4; j++) bfly(v[g + j], v[g + j + 4], W.w[2 * j]);
    }
    bfly1(v[0], v[8]);
#pragma unroll
    for (int j = 1; j < 8; j++) bfly(v[j], v[j + 8], W.w[j]);
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = v[i];
}

#define LAB_FENCE() __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"), __builtin_amdgcn_wave_barrier(), __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront")

__device__ __forceinline__ int pos_in(int k, int line) { return k ^ (line << 2); }
__device__ __forceinline__ int pos_out(int j, int line) { return j ^ (((j >> 6) & 3) << 2) ^ (line << 2); }

__global__ void __launch_bounds__(256, 2) wpass2(const fe *in, fe *out, int log_n, const fe *tw4096, W16 W) {
    __shared__ fe s[4096];
    const size_t n = (size_t)1 << log_n, n2 = n >> 10;
    const size_t j2_0 = xcd_block(blockIdx.x, gridDim.x) * 4;
    in += (size_t)blockIdx.y * n;
    out += (size_t)blockIdx.y * n;
    for (int e = threadIdx.x; e < 4096; e += 256) {
        const int line = e & 3, k1 = e >> 2;
        s[line * 1024 + pos_in(k1, line)] = in[(size_t)k1 * n2 + j2_0 + line];
    }
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    fe *S = s + w * 1024;
    fe x[16];
#pragma unroll
    for (int b = 0; b < 16; b++) x[b] = S[pos_in(lane + 64 * b, w)];
    dft16(x, W);
#pragma unroll
    for (int c = 1; c < 16; c++) x[c] = fe_mul(x[c], tw4096[4 * lane * c]);
    LAB_FENCE();
#pragma unroll
    for (int c = 0; c < 16; c++) S[c * 64 + (lane ^ ((c & 3) << 2))] = x[c];
    LAB_FENCE();
    const int c = lane >> 2, a0 = lane & 3;
#pragma unroll
    for (int a1 = 0; a1 < 16; a1++) x[a1] = S[c * 64 + ((a0 + 4 * a1) ^ ((c & 3) << 2))];
    dft16(x, W);
#pragma unroll
    for (int d0 = 1; d0 < 16; d0++) x[d0] = fe_mul(x[d0], tw4096[64 * a0 * d0]);
    LAB_FENCE();
#pragma unroll
    for (int d0 = 0; d0 < 16; d0++) S[c * 64 + ((4 * d0 + a0) ^ ((c & 3) << 2) ^ (d0 >> 2))] = x[d0];
    LAB_FENCE();
    const int q = a0;
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int b = 0; b < 4; b++) x[4 * r + b] = S[c * 64 + ((16 * q + 4 * r + b) ^ ((c & 3) << 2) ^ q)];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        fe *u = x + 4 * r;
        bfly1(u[0], u[2]);
        bfly1(u[1], u[3]);
        u[3] = fe_mul(u[3], W.w4);
        bfly1(u[0], u[1]);  // X0, X2
        bfly1(u[2], u[3]);  // X1, X3
    }
    LAB_FENCE();
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int j = c + 16 * (4 * q + r);
        S[pos_out(j, w)] = x[4 * r + 0];
        S[pos_out(j + 512, w)] = x[4 * r + 1];
        S[pos_out(j + 256, w)] = x[4 * r + 2];
        S[pos_out(j + 768, w)] = x[4 * r + 3];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 4096; e += 256) {
        const int line = e & 3, j1 = e >> 2;
        out[n2 * (size_t)j1 + j2_0 + line] = s[line * 1024 + pos_out(j1, line)];
    }
}


// ---------------------------------------------------------------- the library pass 2 with switches
// NOSYNC: drop the per-round block barriers (wrong results; measures their cost)
// NOTW:   stage twiddles from registers instead of global loads (wrong results; measures load latency)
template <int LG, bool NOSYNC, bool NOTW>
__device__ __forceinline__ void lab_round(fe *s, const fe *tw4096, fe wfake) {
    constexpr int LOGM = 10, TILE = 4096, M = 1 << LOGM, Q = TILE / 4, h = 1 << (LG - 1);
    using L = Lds<LOGM, TILE>;
    const int q = threadIdx.x;
    const int line = q >> (LOGM - 2), local = q & (M / 4 - 1);
    const int j = local & (h - 1), grp = local >> (LG - 1);
    const int p = L::idx(line, grp * 4 * h + j), ph = L::at(p, h), p2h = L::at(p, 2 * h), p3h = L::at(p, 3 * h);
    const fe w1 = NOTW ? wfake : tw4096[j << (12 - LG)];
    const fe w2 = NOTW ? wfake : tw4096[j << (11 - LG)];
    const fe w3 = NOTW ? wfake : tw4096[(j + h) << (11 - LG)];
    const fe x0 = s[p], x1 = s[ph], x2 = s[p2h], x3 = s[p3h];
    const fe t1 = fe_mul(x1, w1), t3 = fe_mul(x3, w1);
    const fe a0 = fe_add(x0, t1), a1 = fe_sub(x0, t1), a2 = fe_add(x2, t3), a3 = fe_sub(x2, t3);
    const fe u2 = fe_mul(a2, w2), u3 = fe_mul(a3, w3);
    s[p] = fe_add(a0, u2);
    s[p2h] = fe_sub(a0, u2);
    s[ph] = fe_add(a1, u3);
    s[p3h] = fe_sub(a1, u3);
    if (!NOSYNC) __syncthreads();
}
template <bool NOSYNC, bool NOTW>
__global__ void __launch_bounds__(1024, 8) lab_pass2(NttArgs a, fe wfake) {
    extern __shared__ fe s[];
    constexpr int LOGM = 10, TILE = 4096, M = 1 << LOGM, LPB = TILE / M;
    const size_t n = (size_t)1 << a.log_n;
    const size_t n2 = n >> LOGM;
    const size_t j2_0 = xcd_block(blockIdx.x, gridDim.x) * LPB;
    const fe *in = a.in + (size_t)blockIdx.y * a.in_stride;
    for (int e = threadIdx.x; e < TILE; e += 1024) {
        int line = e % LPB, k1 = Lds<LOGM, TILE>::load_k(e / LPB);
        s[Lds<LOGM, TILE>::idx(line, (int)(__brev((unsigned)k1) >> (32 - LOGM)))] = in[(size_t)k1 * n2 + j2_0 + line];
    }
    __syncthreads();
    {
        const fe w4 = a.tw4096[1024];
        using L = Lds<LOGM, TILE>;
        const int q = threadIdx.x;
        const int line = q >> (LOGM - 2), local = q & (M / 4 - 1);
        const int p = L::idx(line, local * 4), p1 = L::at(p, 1), p2 = L::at(p, 2), p3 = L::at(p, 3);
        const fe x0 = s[p], x1 = s[p1], x2 = s[p2], x3 = s[p3];
        const fe a0 = fe_add(x0, x1), a1 = fe_sub(x0, x1), a2 = fe_add(x2, x3);
        const fe a3 = fe_mul(fe_sub(x2, x3), w4);
        s[p] = fe_add(a0, a2);
        s[p2] = fe_sub(a0, a2);
        s[p1] = fe_add(a1, a3);
        s[p3] = fe_sub(a1, a3);
        if (!NOSYNC) __syncthreads();
    }
    lab_round<3, NOSYNC, NOTW>(s, a.tw4096, wfake);
    lab_round<5, NOSYNC, NOTW>(s, a.tw4096, wfake);
    lab_round<7, NOSYNC, NOTW>(s, a.tw4096, wfake);
    lab_round<9, NOSYNC, NOTW>(s, a.tw4096, wfake);
    if (NOSYNC) __syncthreads();
    fe *out = a.out + (size_t)blockIdx.y * a.out_stride;
    for (int e = threadIdx.x; e < TILE; e += 1024) {
        int line = e % LPB, j1 = e / LPB;
        out[n2 * (size_t)j1 + j2_0 + line] = s[Lds<LOGM, TILE>::idx(line, j1)];
    }
}

// ---------------------------------------------------------------- tile-size sweep of the barrier-per-round pass 2
// TILE elements per block (TILE / 1024 lines of 1024), TILE / 4 threads (one radix-4 butterfly each per round)
template <int TILE, int LG>
__device__ __forceinline__ void sw_round(fe *s, const fe *tw4096) {
    constexpr int LOGM = 10, M = 1 << LOGM, h = 1 << (LG - 1);
    using L = Lds<LOGM, TILE>;
    const int q = threadIdx.x;
    const int line = q >> (LOGM - 2), local = q & (M / 4 - 1);
    const int j = local & (h - 1), grp = local >> (LG - 1);
    const int p = L::idx(line, grp * 4 * h + j), ph = L::at(p, h), p2h = L::at(p, 2 * h), p3h = L::at(p, 3 * h);
    const fe w1 = tw4096[j << (12 - LG)];
    const fe w2 = tw4096[j << (11 - LG)];
    const fe w3 = tw4096[(j + h) << (11 - LG)];
    const fe x0 = s[p], x1 = s[ph], x2 = s[p2h], x3 = s[p3h];
    const fe t1 = fe_mul(x1, w1), t3 = fe_mul(x3, w1);
    const fe a0 = fe_add(x0, t1), a1 = fe_sub(x0, t1), a2 = fe_add(x2, t3), a3 = fe_sub(x2, t3);
    const fe u2 = fe_mul(a2, w2), u3 = fe_mul(a3, w3);
    s[p] = fe_add(a0, u2);
    s[p2h] = fe_sub(a0, u2);
    s[ph] = fe_add(a1, u3);
    s[p3h] = fe_sub(a1, u3);
    __syncthreads();
}
template <int TILE>
__global__ void __launch_bounds__(TILE / 4, 8) sw_pass2(NttArgs a) {
    extern __shared__ fe s[];
    constexpr int LOGM = 10, M = 1 << LOGM, LPB = TILE / M, T = TILE / 4;
    const size_t n = (size_t)1 << a.log_n;
    const size_t n2 = n >> LOGM;
    const size_t j2_0 = xcd_block(blockIdx.x, gridDim.x) * LPB;
    const fe *in = a.in + (size_t)blockIdx.y * a.in_stride;
    for (int e = threadIdx.x; e < TILE; e += T) {
        int line = e % LPB, k1 = Lds<LOGM, TILE>::load_k(e / LPB);
        s[Lds<LOGM, TILE>::idx(line, (int)(__brev((unsigned)k1) >> (32 - LOGM)))] = in[(size_t)k1 * n2 + j2_0 + line];
    }
    __syncthreads();
    {
        const fe w4 = a.tw4096[1024];
        using L = Lds<LOGM, TILE>;
        const int q = threadIdx.x;
        const int line = q >> (LOGM - 2), local = q & (M / 4 - 1);
        const int p = L::idx(line, local * 4), p1 = L::at(p, 1), p2 = L::at(p, 2), p3 = L::at(p, 3);
        const fe x0 = s[p], x1 = s[p1], x2 = s[p2], x3 = s[p3];
        const fe a0 = fe_add(x0, x1), a1 = fe_sub(x0, x1), a2 = fe_add(x2, x3);
        const fe a3 = fe_mul(fe_sub(x2, x3), w4);
        s[p] = fe_add(a0, a2);
        s[p2] = fe_sub(a0, a2);
        s[p1] = fe_add(a1, a3);
        s[p3] = fe_sub(a1, a3);
        __syncthreads();
    }
    sw_round<TILE, 3>(s, a.tw4096);
    sw_round<TILE, 5>(s, a.tw4096);
    sw_round<TILE, 7>(s, a.tw4096);
    sw_round<TILE, 9>(s, a.tw4096);
    fe *out = a.out + (size_t)blockIdx.y * a.out_stride;
    for (int e = threadIdx.x; e < TILE; e += T) {
        int line = e % LPB, j1 = e / LPB;
        out[n2 * (size_t)j1 + j2_0 + line] = s[Lds<LOGM, TILE>::idx(line, j1)];
    }
}

// ---------------------------------------------------------------- pass 2 with precomputed-constant twiddles
// Stage twiddles as W sets (tools/ubench/fmul_variants.hpp fe_mul_pre): 64 B per twiddle, 29 % fewer issue
// slots per multiply.  WAVES: launch-bounds waves per SIMD (8: the 64-VGPR budget of the library kernel).
template <int LG, int WAVES, bool FIXEDW = false>
__device__ __forceinline__ void pre_round(fe *s, const WSet *tw, const uint32_t *WF = nullptr) {
    constexpr int LOGM = 10, TILE = 4096, M = 1 << LOGM, h = 1 << (LG - 1);
    using L = Lds<LOGM, TILE>;
    const int q = threadIdx.x;
    const int line = q >> (LOGM - 2), local = q & (M / 4 - 1);
    const int j = local & (h - 1), grp = local >> (LG - 1);
    const int p = L::idx(line, grp * 4 * h + j), ph = L::at(p, h), p2h = L::at(p, 2 * h), p3h = L::at(p, 3 * h);
    const uint32_t *W1 = FIXEDW ? WF : tw[j << (12 - LG)].w;
    const uint32_t *W2 = FIXEDW ? WF : tw[j << (11 - LG)].w;
    const uint32_t *W3 = FIXEDW ? WF : tw[(j + h) << (11 - LG)].w;
    const fe x0 = s[p], x1 = s[ph], x2 = s[p2h], x3 = s[p3h];
    const fe t1 = fe_mul_pre(x1, W1), t3 = fe_mul_pre(x3, W1);
    const fe a0 = fe_add(x0, t1), a1 = fe_sub(x0, t1), a2 = fe_add(x2, t3), a3 = fe_sub(x2, t3);
    const fe u2 = fe_mul_pre(a2, W2), u3 = fe_mul_pre(a3, W3);
    s[p] = fe_add(a0, u2);
    s[p2h] = fe_sub(a0, u2);
    s[ph] = fe_add(a1, u3);
    s[p3h] = fe_sub(a1, u3);
    __syncthreads();
}
template <int WAVES, bool FIXEDW = false>
__global__ void __launch_bounds__(1024, WAVES) pre_pass2(NttArgs a, const WSet *tw) {
    uint32_t WF[16];
#pragma unroll
    for (int k = 0; k < 16; k++) WF[k] = __builtin_amdgcn_readfirstlane(tw[77].w[k]);
    extern __shared__ fe s[];
    constexpr int LOGM = 10, TILE = 4096, M = 1 << LOGM, LPB = TILE / M;
    const size_t n = (size_t)1 << a.log_n;
    const size_t n2 = n >> LOGM;
    const size_t j2_0 = xcd_block(blockIdx.x, gridDim.x) * LPB;
    const fe *in = a.in + (size_t)blockIdx.y * a.in_stride;
    for (int e = threadIdx.x; e < TILE; e += 1024) {
        int line = e % LPB, k1 = Lds<LOGM, TILE>::load_k(e / LPB);
        s[Lds<LOGM, TILE>::idx(line, (int)(__brev((unsigned)k1) >> (32 - LOGM)))] = in[(size_t)k1 * n2 + j2_0 + line];
    }
    __syncthreads();
    {
        using L = Lds<LOGM, TILE>;
        const int q = threadIdx.x;
        const int line = q >> (LOGM - 2), local = q & (M / 4 - 1);
        const int p = L::idx(line, local * 4), p1 = L::at(p, 1), p2 = L::at(p, 2), p3 = L::at(p, 3);
        const fe x0 = s[p], x1 = s[p1], x2 = s[p2], x3 = s[p3];
        const fe a0 = fe_add(x0, x1), a1 = fe_sub(x0, x1), a2 = fe_add(x2, x3);
        const fe a3 = fe_mul_pre(fe_sub(x2, x3), tw[1024].w);
        s[p] = fe_add(a0, a2);
        s[p2] = fe_sub(a0, a2);
        s[p1] = fe_add(a1, a3);
        s[p3] = fe_sub(a1, a3);
        __syncthreads();
    }
    pre_round<3, WAVES, FIXEDW>(s, tw, WF);
    pre_round<5, WAVES, FIXEDW>(s, tw, WF);
    pre_round<7, WAVES, FIXEDW>(s, tw, WF);
    pre_round<9, WAVES, FIXEDW>(s, tw, WF);
    fe *out = a.out + (size_t)blockIdx.y * a.out_stride;
    for (int e = threadIdx.x; e < TILE; e += 1024) {
        int line = e % LPB, j1 = e / LPB;
        out[n2 * (size_t)j1 + j2_0 + line] = s[Lds<LOGM, TILE>::idx(line, j1)];
    }
}

// ---------------------------------------------------------------- uniform-twiddle rounds
// Rounds with half-size h <= 16 remap threads to butterflies so that every wave shares one twiddle index j:
// the twiddle's W set is wave-uniform (scalar loads into SGPRs) and the multiply is the precomputed-
// constant form.  Rounds h = 64, 256 keep the library mapping and plain multiplies.
__device__ __forceinline__ void col3s(uint64_t &a, uint32_t &h, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                                      uint32_t x2, uint32_t y2) {
    uint64_t k0, k1, k2, kd;
    asm("v_mad_u64_u32 %0, %2, %6, %7, %0\n\t"
        "v_mad_u64_u32 %0, %3, %8, %9, %0\n\t"
        "v_mad_u64_u32 %0, %4, %10, %11, %0\n\t"
        "v_addc_co_u32 %1, %5, 0, 0, %2\n\t"
        "v_addc_co_u32 %1, %5, %1, 0, %3\n\t"
        "v_addc_co_u32 %1, %5, %1, 0, %4"
        : "+v"(a), "=&v"(h), "=&s"(k0), "=&s"(k1), "=&s"(k2), "=&s"(kd)
        : "v"(x0), "s"(y0), "v"(x1), "s"(y1), "v"(x2), "s"(y2));
}
__device__ __forceinline__ void col4s(uint64_t &a, uint32_t &h, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                                      uint32_t x2, uint32_t y2, uint32_t x3, uint32_t y3) {
    uint64_t k0, k1, k2, k3, kd;
    asm("v_mad_u64_u32 %0, %2, %7, %8, %0\n\t"
        "v_mad_u64_u32 %0, %3, %9, %10, %0\n\t"
        "v_mad_u64_u32 %0, %4, %11, %12, %0\n\t"
        "v_mad_u64_u32 %0, %5, %13, %14, %0\n\t"
        "v_addc_co_u32 %1, %6, 0, 0, %2\n\t"
        "v_addc_co_u32 %1, %6, %1, 0, %3\n\t"
        "v_addc_co_u32 %1, %6, %1, 0, %4\n\t"
        "v_addc_co_u32 %1, %6, %1, 0, %5"
        : "+v"(a), "=&v"(h), "=&s"(k0), "=&s"(k1), "=&s"(k2), "=&s"(k3), "=&s"(kd)
        : "v"(x0), "s"(y0), "v"(x1), "s"(y1), "v"(x2), "s"(y2), "v"(x3), "s"(y3));
}
struct WS {
    uint32_t w[16];
};
// W set of a wave-uniform twiddle, loaded with scalar loads
__device__ __forceinline__ WS load_ws(const WSet *__restrict__ tw, int idx) {
    WS r;
#pragma unroll
    for (int k = 0; k < 16; k++) r.w[k] = __builtin_amdgcn_readfirstlane(tw[idx].w[k]);
    return r;
}
__device__ __forceinline__ fe fe_mul_ws(fe A, const WS &W) {
    const uint32_t x0 = lo32(A.lo), x1 = hi32(A.lo), x2 = lo32(A.hi), x3 = hi32(A.hi);
    uint32_t r0, r1, r2, r3;
    uint64_t a;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(a), "=s"(*(uint64_t[1]){}) : "v"(x0), "s"(W.w[0]));
    uint32_t h = 0;
    col3s(a, h, x1, W.w[1], x2, W.w[2], x3, W.w[3]);               ZK_SHIFT2(a, h, r0);
    col4s(a, h, x0, W.w[4], x1, W.w[5], x2, W.w[6], x3, W.w[7]);   ZK_SHIFT2(a, h, r1);
    col4s(a, h, x0, W.w[8], x1, W.w[9], x2, W.w[10], x3, W.w[11]); ZK_SHIFT2(a, h, r2);
    col4s(a, h, x0, W.w[12], x1, W.w[13], x2, W.w[14], x3, W.w[15]); ZK_SHIFT2(a, h, r3);
    return pre_fold(r0, r1, r2, r3, (uint32_t)a, (uint32_t)(a >> 32));
}
template <int LG>
__device__ __forceinline__ void uni_round(fe *s, const WSet *__restrict__ tw) {
    constexpr int LOGM = 10, TILE = 4096, M = 1 << LOGM, h = 1 << (LG - 1), LH = LG - 1;
    using L = Lds<LOGM, TILE>;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
    const int j = w >> (4 - LH);
    const int pidx = ((w & ((16 >> LH) - 1)) << 6) | l;
    const int line = pidx >> (8 - LH), grp = pidx & ((256 >> LH) - 1);
    const int p = L::idx(line, grp * 4 * h + j), ph = L::at(p, h), p2h = L::at(p, 2 * h), p3h = L::at(p, 3 * h);
    const WS W1 = load_ws(tw, j << (12 - LG));
    const fe x0 = s[p], x1 = s[ph], x2 = s[p2h], x3 = s[p3h];
    const fe t1 = fe_mul_ws(x1, W1), t3 = fe_mul_ws(x3, W1);
    const fe a0 = fe_add(x0, t1), a1 = fe_sub(x0, t1), a2 = fe_add(x2, t3), a3 = fe_sub(x2, t3);
    const WS W2 = load_ws(tw, j << (11 - LG));
    const fe u2 = fe_mul_ws(a2, W2);
    const WS W3 = load_ws(tw, (j + h) << (11 - LG));
    const fe u3 = fe_mul_ws(a3, W3);
    s[p] = fe_add(a0, u2);
    s[p2h] = fe_sub(a0, u2);
    s[ph] = fe_add(a1, u3);
    s[p3h] = fe_sub(a1, u3);
    __syncthreads();
}
__global__ void __launch_bounds__(1024, 8) uni_pass2(NttArgs a, const WSet *__restrict__ tw) {
    extern __shared__ fe s[];
    constexpr int LOGM = 10, TILE = 4096, M = 1 << LOGM, LPB = TILE / M;
    const size_t n = (size_t)1 << a.log_n;
    const size_t n2 = n >> LOGM;
    const size_t j2_0 = xcd_block(blockIdx.x, gridDim.x) * LPB;
    const fe *in = a.in + (size_t)blockIdx.y * a.in_stride;
    for (int e = threadIdx.x; e < TILE; e += 1024) {
        int line = e % LPB, k1 = Lds<LOGM, TILE>::load_k(e / LPB);
        s[Lds<LOGM, TILE>::idx(line, (int)(__brev((unsigned)k1) >> (32 - LOGM)))] = in[(size_t)k1 * n2 + j2_0 + line];
    }
    __syncthreads();
    {
        using L = Lds<LOGM, TILE>;
        const int q = threadIdx.x;
        const int line = q >> (LOGM - 2), local = q & (M / 4 - 1);
        const int p = L::idx(line, local * 4), p1 = L::at(p, 1), p2 = L::at(p, 2), p3 = L::at(p, 3);
        const WS W4 = load_ws(tw, 1024);
        const fe x0 = s[p], x1 = s[p1], x2 = s[p2], x3 = s[p3];
        const fe a0 = fe_add(x0, x1), a1 = fe_sub(x0, x1), a2 = fe_add(x2, x3);
        const fe a3 = fe_mul_ws(fe_sub(x2, x3), W4);
        s[p] = fe_add(a0, a2);
        s[p2] = fe_sub(a0, a2);
        s[p1] = fe_add(a1, a3);
        s[p3] = fe_sub(a1, a3);
        __syncthreads();
    }
    uni_round<3>(s, tw);
    uni_round<5>(s, tw);
    lab_round<7, false, false>(s, a.tw4096, fe_zero());
    lab_round<9, false, false>(s, a.tw4096, fe_zero());
    fe *out = a.out + (size_t)blockIdx.y * a.out_stride;
    for (int e = threadIdx.x; e < TILE; e += 1024) {
        int line = e % LPB, j1 = e / LPB;
        out[n2 * (size_t)j1 + j2_0 + line] = s[Lds<LOGM, TILE>::idx(line, j1)];
    }
}

// ---------------------------------------------------------------- uniform-twiddle rounds on a re-swizzled tile
// sw(x) = x ^ bits 4-7 ^ bits 8-9 (folded into bits 0-3): conflict-free for the remapped rounds h = 4, 16
// as well as the library mapping of h = 1, 64, 256 and the load / store phases (host model).
struct NL {
    __device__ __forceinline__ static int sw(int x) { return x ^ ((x >> 4) & 15) ^ ((x >> 8) & 3); }
    __device__ __forceinline__ static int idx(int line, int pos) { return line * 1024 + (sw(pos) ^ ((line & 3) << 2)); }
    __device__ __forceinline__ static int at(int p, int d) { return p ^ sw(d); }
};
template <int LG, bool UNI>
__device__ __forceinline__ void nl_round(fe *s, const WSet *__restrict__ tw, const fe *tw4096) {
    constexpr int h = 1 << (LG - 1), LH = LG - 1;
    int line, grp, j;
    if constexpr (UNI) {
        const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
        j = w >> (4 - LH);
        const int pidx = ((w & ((16 >> LH) - 1)) << 6) | l;
        line = pidx >> (8 - LH);
        grp = pidx & ((256 >> LH) - 1);
    } else {
        const int q = threadIdx.x;
        line = q >> 8;
        const int local = q & 255;
        j = local & (h - 1);
        grp = local >> LH;
    }
    const int p = NL::idx(line, grp * 4 * h + j), ph = NL::at(p, h), p2h = NL::at(p, 2 * h), p3h = NL::at(p, 3 * h);
    const fe x0 = s[p], x1 = s[ph], x2 = s[p2h], x3 = s[p3h];
    fe t1, t3, u2, u3, a0, a1, a2, a3;
    if constexpr (UNI) {
        const WS W1 = load_ws(tw, j << (12 - LG));
        t1 = fe_mul_ws(x1, W1);
        t3 = fe_mul_ws(x3, W1);
        a0 = fe_add(x0, t1); a1 = fe_sub(x0, t1); a2 = fe_add(x2, t3); a3 = fe_sub(x2, t3);
        const WS W2 = load_ws(tw, j << (11 - LG));
        u2 = fe_mul_ws(a2, W2);
        const WS W3 = load_ws(tw, (j + h) << (11 - LG));
        u3 = fe_mul_ws(a3, W3);
    } else {
        const fe w1 = tw4096[j << (12 - LG)], w2 = tw4096[j << (11 - LG)], w3 = tw4096[(j + h) << (11 - LG)];
        t1 = fe_mul(x1, w1);
        t3 = fe_mul(x3, w1);
        a0 = fe_add(x0, t1); a1 = fe_sub(x0, t1); a2 = fe_add(x2, t3); a3 = fe_sub(x2, t3);
        u2 = fe_mul(a2, w2);
        u3 = fe_mul(a3, w3);
    }
    s[p] = fe_add(a0, u2);
    s[p2h] = fe_sub(a0, u2);
    s[ph] = fe_add(a1, u3);
    s[p3h] = fe_sub(a1, u3);
    __syncthreads();
}
template <bool UNI>
__global__ void __launch_bounds__(1024, 8) nl_pass2(NttArgs a, const WSet *__restrict__ tw) {
    extern __shared__ fe s[];
    constexpr int LOGM = 10, TILE = 4096, LPB = 4;
    const size_t n = (size_t)1 << a.log_n;
    const size_t n2 = n >> LOGM;
    const size_t j2_0 = xcd_block(blockIdx.x, gridDim.x) * LPB;
    const fe *in = a.in + (size_t)blockIdx.y * a.in_stride;
    for (int e = threadIdx.x; e < TILE; e += 1024) {
        int line = e % LPB, v = e / LPB, k1 = ((v & 3) << 8) | (v >> 2);
        s[NL::idx(line, (int)(__brev((unsigned)k1) >> (32 - LOGM)))] = in[(size_t)k1 * n2 + j2_0 + line];
    }
    __syncthreads();
    {
        const int q = threadIdx.x;
        const int line = q >> 8, local = q & 255;
        const int p = NL::idx(line, local * 4), p1 = NL::at(p, 1), p2 = NL::at(p, 2), p3 = NL::at(p, 3);
        const fe x0 = s[p], x1 = s[p1], x2 = s[p2], x3 = s[p3];
        const fe a0 = fe_add(x0, x1), a1 = fe_sub(x0, x1), a2 = fe_add(x2, x3);
        fe a3;
        if constexpr (UNI) a3 = fe_mul_ws(fe_sub(x2, x3), load_ws(tw, 1024));
        else a3 = fe_mul(fe_sub(x2, x3), a.tw4096[1024]);
        s[p] = fe_add(a0, a2);
        s[p2] = fe_sub(a0, a2);
        s[p1] = fe_add(a1, a3);
        s[p3] = fe_sub(a1, a3);
        __syncthreads();
    }
    nl_round<3, UNI>(s, tw, a.tw4096);
    nl_round<5, UNI>(s, tw, a.tw4096);
    nl_round<7, false>(s, tw, a.tw4096);
    nl_round<9, false>(s, tw, a.tw4096);
    fe *out = a.out + (size_t)blockIdx.y * a.out_stride;
    for (int e = threadIdx.x; e < TILE; e += 1024) {
        int line = e % LPB, j1 = e / LPB;
        out[n2 * (size_t)j1 + j2_0 + line] = s[NL::idx(line, j1)];
    }
}
// ---------------------------------------------------------------- harness
static fe h_pow(fe b, uint64_t e) {
    fe r = fe_one();
    while (e) {
        if (e & 1) r = fe_mul(r, b);
        b = fe_mul(b, b);
        e >>= 1;
    }
    return r;
}

int main(int argc, char **argv) {
    const int log_n = 20, batch = argc > 1 ? atoi(argv[1]) : 28;
    const size_t n = (size_t)1 << log_n, tot = n * batch;
    std::vector<fe> h(tot);
    uint64_t st = 88172645463325252ull;
    for (auto &v : h) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17; v.lo = st;
        st ^= st << 13; st ^= st >> 7; st ^= st << 17; v.hi = st >> 1;
    }
    const fe w4096 = h_root_of_unity(12);
    std::vector<fe> tw(4096);
    tw[0] = fe_one();
    for (int i = 1; i < 4096; i++) tw[i] = fe_mul(tw[i - 1], w4096);
    W16 W;
    for (int i = 0; i < 8; i++) W.w[i] = tw[256 * i];
    W.w4 = tw[1024];
    fe *din, *dout0, *dout1, *dtw;
    (void)hipMalloc(&din, tot * sizeof(fe));
    (void)hipMalloc(&dout0, tot * sizeof(fe));
    (void)hipMalloc(&dout1, tot * sizeof(fe));
    (void)hipMalloc(&dtw, 4096 * sizeof(fe));
    (void)hipMemcpy(din, h.data(), tot * sizeof(fe), hipMemcpyHostToDevice);
    (void)hipMemcpy(dtw, tw.data(), 4096 * sizeof(fe), hipMemcpyHostToDevice);
    (void)hipMemset(dout0, 0, tot * sizeof(fe));
    (void)hipMemset(dout1, 0xff, tot * sizeof(fe));

    NttArgs a;
    memset(&a, 0, sizeof a);
    a.in = din;
    a.out = dout0;
    a.in_stride = n;
    a.out_stride = n;
    a.tw4096 = dtw;
    a.log_n = log_n;
    a.ncos = 1;
    const size_t sh = Lds<10, 4096>::bytes();
    (void)hipFuncSetAttribute((const void *)ntt_pass2<10, 4096>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    auto base = [&] { hipLaunchKernelGGL((ntt_pass2<10, 4096>), dim3(n / 1024 / 4, batch), dim3(1024), sh, 0, a); };
    auto wv = [&] { hipLaunchKernelGGL(wpass2, dim3(n / 1024 / 4, batch), dim3(256), 0, 0, din, dout1, log_n, dtw, W); };
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto timeit = [&](auto f) {
        f();
        (void)hipDeviceSynchronize();
        float best = 1e9;
        for (int r = 0; r < 5; r++) {
            (void)hipEventRecord(e0);
            f();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            best = std::min(best, ms);
        }
        return best;
    };

    for (int v = 0; v < 4; v++) {
        const bool ns = v & 1, nt = v & 2;
        const void *k = ns ? (nt ? (const void *)lab_pass2<true, true> : (const void *)lab_pass2<true, false>)
                           : (nt ? (const void *)lab_pass2<false, true> : (const void *)lab_pass2<false, false>);
        (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
        NttArgs b = a;
        b.out = dout1;
        const fe wf = tw[77];
        auto f = [&] {
            if (v == 0) hipLaunchKernelGGL((lab_pass2<false, false>), dim3(n / 4096, batch), dim3(1024), sh, 0, b, wf);
            if (v == 1) hipLaunchKernelGGL((lab_pass2<true, false>), dim3(n / 4096, batch), dim3(1024), sh, 0, b, wf);
            if (v == 2) hipLaunchKernelGGL((lab_pass2<false, true>), dim3(n / 4096, batch), dim3(1024), sh, 0, b, wf);
            if (v == 3) hipLaunchKernelGGL((lab_pass2<true, true>), dim3(n / 4096, batch), dim3(1024), sh, 0, b, wf);
        };
        printf("lab pass2 nosync=%d notw=%d: %.3f ms\n", (int)ns, (int)nt, timeit(f));
    }

    {
        NttArgs b = a;
        b.out = dout1;
        std::vector<fe> ref(tot), got(tot);
        hipLaunchKernelGGL((ntt_pass2<10, 4096>), dim3(n / 4096, batch), dim3(1024), sh, 0, a);
        (void)hipMemcpy(ref.data(), dout0, tot * sizeof(fe), hipMemcpyDeviceToHost);
        auto sweep = [&](auto kern, int tile, size_t shb) {
            (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shb);
            auto f = [&] { hipLaunchKernelGGL(kern, dim3(n / tile, batch), dim3(tile / 4), shb, 0, b); };
            const float t = timeit(f);
            (void)hipMemcpy(got.data(), dout1, tot * sizeof(fe), hipMemcpyDeviceToHost);
            size_t bad = 0;
            for (size_t i = 0; i < tot; i++) bad += !fe_eq(ref[i], got[i]);
            printf("tile %4d (%d threads, %d lines): %.3f ms, mismatches %zu\n", tile, tile / 4, tile / 1024, t, bad);
        };
        sweep(sw_pass2<4096>, 4096, Lds<10, 4096>::bytes());
        sweep(sw_pass2<2048>, 2048, Lds<10, 2048>::bytes());
        sweep(sw_pass2<1024>, 1024, Lds<10, 1024>::bytes());
        sweep(sw_pass2<8192>, 8192, Lds<10, 8192>::bytes());
    }

    {
        std::vector<WSet> hw(4096);
        for (int i = 0; i < 4096; i++) hw[i] = make_wset(tw[i]);
        WSet *dws;
        (void)hipMalloc(&dws, 4096 * sizeof(WSet));
        (void)hipMemcpy(dws, hw.data(), 4096 * sizeof(WSet), hipMemcpyHostToDevice);
        NttArgs b = a;
        b.out = dout1;
        std::vector<fe> ref(tot), got(tot);
        hipLaunchKernelGGL((ntt_pass2<10, 4096>), dim3(n / 4096, batch), dim3(1024), sh, 0, a);
        (void)hipMemcpy(ref.data(), dout0, tot * sizeof(fe), hipMemcpyDeviceToHost);
        auto run_pre = [&](auto kern, const char *name) {
            (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
            auto f = [&] { hipLaunchKernelGGL(kern, dim3(n / 4096, batch), dim3(1024), sh, 0, b, (const WSet *)dws); };
            const float t = timeit(f);
            (void)hipMemcpy(got.data(), dout1, tot * sizeof(fe), hipMemcpyDeviceToHost);
            size_t bad = 0;
            for (size_t i = 0; i < tot; i++) bad += !fe_eq(ref[i], got[i]);
            printf("%s: %.3f ms, mismatches %zu\n", name, t, bad);
        };
        run_pre(pre_pass2<8>, "pre-twiddle pass2, 8 waves/SIMD");
        run_pre(pre_pass2<4>, "pre-twiddle pass2, 4 waves/SIMD");
        run_pre(pre_pass2<8, true>, "pre-twiddle pass2, 8 waves/SIMD, one W set in SGPRs (timing only)");
        run_pre(uni_pass2, "uniform-twiddle rounds h<=16 (scalar W sets), plain h=64,256");
        run_pre(nl_pass2<false>, "new swizzle, library mapping and multiplies");
        run_pre(nl_pass2<true>, "new swizzle, uniform-twiddle rounds h<=16");
    }
    const float t0 = timeit(base), t1 = timeit(wv);
    std::vector<fe> o0(tot), o1(tot);
    (void)hipMemcpy(o0.data(), dout0, tot * sizeof(fe), hipMemcpyDeviceToHost);
    (void)hipMemcpy(o1.data(), dout1, tot * sizeof(fe), hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (size_t i = 0; i < tot; i++) bad += !fe_eq(o0[i], o1[i]);
    printf("pass2 1024-pt lines, %d x 2^%d: library %.3f ms, wave-per-line %.3f ms (%.2fx), mismatches %zu\n", batch, log_n, t0, t1,
           t0 / t1, bad);
    printf("err: %s\n", hipGetErrorString(hipGetLastError()));
    return bad != 0;
}
