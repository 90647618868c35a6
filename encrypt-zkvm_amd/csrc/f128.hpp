// f128.hpp -- the winterfell f128 prime field, p = 2^128 - 45*2^40 + 1, for gfx950 and host.
//
// Canonical representation in [0, p), stored as two little-endian u64 halves: exactly the
// 16-byte wire format of winter-math `f128::BaseElement` (prover/src/lib.rs:4).
//
// Device multiply: 4x4 schoolbook on 32-bit limbs with v_mad_u64_u32 (16 partial products),
// then two folds of the high half with 2^128 = C (mod p), C = 45*2^40 - 1, and one conditional
// subtraction.  Everything is branch-free so a wavefront never diverges on data.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "addsub_asm.hpp"

#define ZK_HD __host__ __device__ __forceinline__

struct fe {
    uint64_t lo, hi;
};

static constexpr uint64_t ZK_P_LO = 0xffffd30000000001ULL;  // p mod 2^64
static constexpr uint64_t ZK_P_HI = 0xffffffffffffffffULL;  // p >> 64
static constexpr uint64_t ZK_C = 0x2cffffffffffULL;         // 2^128 - p = 45*2^40 - 1

ZK_HD fe fe_make(uint64_t lo, uint64_t hi = 0) { return fe{lo, hi}; }
ZK_HD fe fe_zero() { return fe{0, 0}; }
ZK_HD fe fe_one() { return fe{1, 0}; }
ZK_HD bool fe_eq(fe a, fe b) { return a.lo == b.lo && a.hi == b.hi; }
ZK_HD bool fe_is_zero(fe a) { return (a.lo | a.hi) == 0; }

ZK_HD uint32_t lo32(uint64_t v) { return (uint32_t)v; }
ZK_HD uint32_t hi32(uint64_t v) { return (uint32_t)(v >> 32); }
ZK_HD uint64_t join32(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }

// a + b mod p on 32-bit carry chains.  s = a + b (129 bits); s >= p  <=>  carry(a+b) or
// carry(s + C), and then s - p = s + C (mod 2^128).
ZK_HD fe fe_add(fe a, fe b) {
    uint32_t c, d, c1, c2;
    const uint32_t s0 = __builtin_addc(lo32(a.lo), lo32(b.lo), 0u, &c);
    const uint32_t s1 = __builtin_addc(hi32(a.lo), hi32(b.lo), c, &c);
    const uint32_t s2 = __builtin_addc(lo32(a.hi), lo32(b.hi), c, &c);
    const uint32_t s3 = __builtin_addc(hi32(a.hi), hi32(b.hi), c, &c1);
    const uint32_t t0 = __builtin_addc(s0, 0xffffffffu, 0u, &d);
    const uint32_t t1 = __builtin_addc(s1, 0x2cffu, d, &d);
    const uint32_t t2 = __builtin_addc(s2, 0u, d, &d);
    const uint32_t t3 = __builtin_addc(s3, 0u, d, &c2);
    const uint32_t m = 0u - ((c1 | c2) & 1u);
    return fe{join32((t0 & m) | (s0 & ~m), (t1 & m) | (s1 & ~m)), join32((t2 & m) | (s2 & ~m), (t3 & m) | (s3 & ~m))};
}

// a - b mod p.  d = a - b (mod 2^128); on borrow the value is d - 2^128 = d - C - p, i.e. d - C.
ZK_HD fe fe_sub(fe a, fe b) {
    uint32_t bw, e;
    const uint32_t d0 = __builtin_subc(lo32(a.lo), lo32(b.lo), 0u, &bw);
    const uint32_t d1 = __builtin_subc(hi32(a.lo), hi32(b.lo), bw, &bw);
    const uint32_t d2 = __builtin_subc(lo32(a.hi), lo32(b.hi), bw, &bw);
    const uint32_t d3 = __builtin_subc(hi32(a.hi), hi32(b.hi), bw, &bw);
    const uint32_t m = 0u - (bw & 1u);
    const uint32_t r0 = __builtin_subc(d0, m, 0u, &e);
    const uint32_t r1 = __builtin_subc(d1, m & 0x2cffu, e, &e);
    const uint32_t r2 = __builtin_subc(d2, 0u, e, &e);
    const uint32_t r3 = __builtin_subc(d3, 0u, e, &e);
    return fe{join32(r0, r1), join32(r2, r3)};
}

ZK_HD fe fe_neg(fe a) { return fe_sub(fe_zero(), a); }

// ---- lazy (partially reduced) forms for the NTT butterflies: values < 2^128, congruent mod p, not
// necessarily canonical.  Contract: the FIRST operand may be any value < 2^128, the SECOND must be
// canonical (< p) -- in a radix-4 butterfly the second operands are multiply outputs, which are canonical.
//   fe_add_lazy: s = a + b < 2^128 + p; on carry s - 2^128 + C = s - p < 2^128 (one fold, no compare with p).
//   fe_sub (above) already satisfies it: no borrow gives a - b < 2^128; a borrow means a < b < p, and
//   a - b + p lies in (0, p).
// A lazy value goes to memory only through fe_canon or a multiply (whose output is canonical).
ZK_HD fe fe_add_lazy(fe a, fe b) {
    uint32_t c, d;
    const uint32_t s0 = __builtin_addc(lo32(a.lo), lo32(b.lo), 0u, &c);
    const uint32_t s1 = __builtin_addc(hi32(a.lo), hi32(b.lo), c, &c);
    const uint32_t s2 = __builtin_addc(lo32(a.hi), lo32(b.hi), c, &c);
    const uint32_t s3 = __builtin_addc(hi32(a.hi), hi32(b.hi), c, &c);
    const uint32_t m = 0u - (c & 1u);  // C = 0x2cff_ffffffff on carry
    const uint32_t t0 = __builtin_addc(s0, m, 0u, &d);
    const uint32_t t1 = __builtin_addc(s1, m & 0x2cffu, d, &d);
    const uint32_t t2 = __builtin_addc(s2, 0u, d, &d);
    const uint32_t t3 = s3 + d;
    return fe{join32(t0, t1), join32(t2, t3)};
}
// the canonical representative of a value < 2^128: v >= p  <=>  carry(v + C), and then v - p = v + C mod 2^128
ZK_HD fe fe_canon(fe v) {
    uint32_t d;
    const uint32_t t0 = __builtin_addc(lo32(v.lo), 0xffffffffu, 0u, &d);
    const uint32_t t1 = __builtin_addc(hi32(v.lo), 0x2cffu, d, &d);
    const uint32_t t2 = __builtin_addc(lo32(v.hi), 0u, d, &d);
    const uint32_t t3 = __builtin_addc(hi32(v.hi), 0u, d, &d);
    const uint32_t m = 0u - (d & 1u);
    return fe{join32((t0 & m) | (lo32(v.lo) & ~m), (t1 & m) | (hi32(v.lo) & ~m)),
              join32((t2 & m) | (lo32(v.hi) & ~m), (t3 & m) | (hi32(v.hi) & ~m))};
}

// r[0..8) = x[0..4) * y[0..4) (operand scanning; each step fits one v_mad_u64_u32 + carry add)
ZK_HD void mul_4x4(const uint32_t x[4], const uint32_t y[4], uint32_t r[8]) {
    uint64_t t;
    uint32_t c;
    t = (uint64_t)x[0] * y[0];
    r[0] = lo32(t);
    c = hi32(t);
    t = (uint64_t)x[0] * y[1] + c;
    r[1] = lo32(t);
    c = hi32(t);
    t = (uint64_t)x[0] * y[2] + c;
    r[2] = lo32(t);
    c = hi32(t);
    t = (uint64_t)x[0] * y[3] + c;
    r[3] = lo32(t);
    r[4] = hi32(t);
#pragma unroll
    for (int i = 1; i < 4; i++) {
        c = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            t = (uint64_t)x[i] * y[j] + (uint64_t)r[i + j] + c;
            r[i + j] = lo32(t);
            c = hi32(t);
        }
        r[i + 4] = c;
    }
}

// Reduction used by the device multiply (shared with the host so the unit test covers it).
// With C = 2^128 - p = 0x2D00 * 2^32 - 1:  x*C = (x * 0x2D00) << 32 - x, so each fold is a short
// multiply by the 14-bit constant K = 0x2D00 plus add/subtract carry chains:
//   S = L - H + (H*K) << 32          (0 <= S < 2^175, computed mod 2^192)
//   T = S_lo - S_hi + (S_hi*K) << 32 (S_hi < 2^47; T < 2^128 + 2^93, bit 128 = tc)
// then one conditional subtract of p (add C, keep on carry).
ZK_HD fe reduce_fold(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t r4, uint32_t r5, uint32_t r6,
                     uint32_t r7) {
    const uint32_t K = 0x2d00u;
    uint64_t q = (uint64_t)r4 * K;
    const uint32_t q0 = lo32(q);
    q = (uint64_t)r5 * K + (q >> 32);
    const uint32_t q1 = lo32(q);
    q = (uint64_t)r6 * K + (q >> 32);
    const uint32_t q2 = lo32(q);
    q = (uint64_t)r7 * K + (q >> 32);
    const uint32_t q3 = lo32(q), q4 = hi32(q);
    uint32_t b, c;
    const uint32_t d0 = __builtin_subc(r0, r4, 0u, &b);
    const uint32_t d1 = __builtin_subc(r1, r5, b, &b);
    const uint32_t d2 = __builtin_subc(r2, r6, b, &b);
    const uint32_t d3 = __builtin_subc(r3, r7, b, &b);
    const uint32_t dm = 0u - b;  // sign extension of L - H into limbs 4, 5
    const uint32_t s1 = __builtin_addc(d1, q0, 0u, &c);
    const uint32_t s2 = __builtin_addc(d2, q1, c, &c);
    const uint32_t s3 = __builtin_addc(d3, q2, c, &c);
    const uint32_t s4 = __builtin_addc(dm, q3, c, &c);
    const uint32_t s5 = dm + q4 + c;
    uint64_t p = (uint64_t)s4 * K;
    const uint32_t p0 = lo32(p);
    p = (uint64_t)s5 * K + (p >> 32);
    const uint32_t p1 = lo32(p), p2 = hi32(p);
    const uint32_t e0 = __builtin_subc(d0, s4, 0u, &b);
    const uint32_t e1 = __builtin_subc(s1, s5, b, &b);
    const uint32_t e2 = __builtin_subc(s2, 0u, b, &b);
    const uint32_t e3 = __builtin_subc(s3, 0u, b, &b);
    const uint32_t t0 = e0;
    const uint32_t t1 = __builtin_addc(e1, p0, 0u, &c);
    const uint32_t t2 = __builtin_addc(e2, p1, c, &c);
    const uint32_t t3 = __builtin_addc(e3, p2, c, &c);
    const uint32_t tc = c ^ b;  // T >= 0, so a borrow out always meets a carry out
    // result = (tc | carry(T + C)) ? T + C : T
    uint32_t cy, uc;
    const uint32_t u0 = __builtin_addc(t0, 0xffffffffu, 0u, &cy);
    const uint32_t u1 = __builtin_addc(t1, 0x2cffu, cy, &cy);
    const uint32_t u2 = __builtin_addc(t2, 0u, cy, &cy);
    const uint32_t u3 = __builtin_addc(t3, 0u, cy, &uc);
    const uint32_t m = 0u - ((tc | uc) & 1u);
    fe res;
    res.lo = ((uint64_t)((u1 & m) | (t1 & ~m)) << 32) | ((u0 & m) | (t0 & ~m));
    res.hi = ((uint64_t)((u3 & m) | (t3 & ~m)) << 32) | ((u2 & m) | (t2 & ~m));
    return res;
}

// the device multiply's algorithm in portable form (host unit test: schoolbook + reduce_fold)
ZK_HD fe fe_mul_limbs(fe a, fe b) {
    uint32_t x[4] = {lo32(a.lo), hi32(a.lo), lo32(a.hi), hi32(a.hi)};
    uint32_t y[4] = {lo32(b.lo), hi32(b.lo), lo32(b.hi), hi32(b.hi)};
    uint32_t r[8];
    mul_4x4(x, y, r);
    return reduce_fold(r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
}

// ---- gfx950 device multiply: product scanning with v_mad_u64_u32 hardware carry-outs ----
// Same algorithm as fe_mul_limbs (schoolbook + two folds with C = 2^128 - p), hand-scheduled:
// (DESIGN.md "Field multiply").
// One column of a product-scanning multiply: a += sum x_i*y_i (64-bit); h := sum of the carry-outs
// (h is the high word of the next column's accumulator).  All MADs first, carry-outs to distinct
// SGPR pairs, then the carry adds: gfx950 needs 2 wait states between a VALU writing an SGPR and a
// VALU reading it as carry-in, which the other instructions (or an s_nop) provide.
__device__ __forceinline__ void col1(uint64_t &a, uint32_t &h, uint32_t x0, uint32_t y0) {
    uint64_t k0, kd;
    asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\t"
        "s_nop 1\n\t"
        "v_addc_co_u32 %1, %3, 0, 0, %2"
        : "+v"(a), "=&v"(h), "=&s"(k0), "=&s"(kd) : "v"(x0), "v"(y0));
}
__device__ __forceinline__ void col2(uint64_t &a, uint32_t &h, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1) {
    uint64_t k0, k1, kd;
    asm("v_mad_u64_u32 %0, %2, %5, %6, %0\n\t"
        "v_mad_u64_u32 %0, %3, %7, %8, %0\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32 %1, %4, 0, 0, %2\n\t"
        "v_addc_co_u32 %1, %4, %1, 0, %3"
        : "+v"(a), "=&v"(h), "=&s"(k0), "=&s"(k1), "=&s"(kd) : "v"(x0), "v"(y0), "v"(x1), "v"(y1));
}
__device__ __forceinline__ void col3(uint64_t &a, uint32_t &h, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                                     uint32_t x2, uint32_t y2) {
    uint64_t k0, k1, k2, kd;
    asm("v_mad_u64_u32 %0, %2, %6, %7, %0\n\t"
        "v_mad_u64_u32 %0, %3, %8, %9, %0\n\t"
        "v_mad_u64_u32 %0, %4, %10, %11, %0\n\t"
        "v_addc_co_u32 %1, %5, 0, 0, %2\n\t"
        "v_addc_co_u32 %1, %5, %1, 0, %3\n\t"
        "v_addc_co_u32 %1, %5, %1, 0, %4"
        : "+v"(a), "=&v"(h), "=&s"(k0), "=&s"(k1), "=&s"(k2), "=&s"(kd)
        : "v"(x0), "v"(y0), "v"(x1), "v"(y1), "v"(x2), "v"(y2));
}
__device__ __forceinline__ void col4(uint64_t &a, uint32_t &h, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
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
        : "v"(x0), "v"(y0), "v"(x1), "v"(y1), "v"(x2), "v"(y2), "v"(x3), "v"(y3));
}
#define ZK_SHIFT(a, h, out) do { out = (uint32_t)(a); a = ((a) >> 32) | ((uint64_t)(h) << 32); h = 0; } while (0)

// full 256-bit product r[0..8) of two 128-bit values
__device__ __forceinline__ void mul_wide(fe A, fe Bv, uint32_t r[8]) {
    const uint32_t x0 = lo32(A.lo), x1 = hi32(A.lo), x2 = lo32(A.hi), x3 = hi32(A.hi);
    const uint32_t y0 = lo32(Bv.lo), y1 = hi32(Bv.lo), y2 = lo32(Bv.hi), y3 = hi32(Bv.hi);
    uint32_t &r0 = r[0], &r1 = r[1], &r2 = r[2], &r3 = r[3], &r4 = r[4], &r5 = r[5], &r6 = r[6], &r7 = r[7];
    uint64_t a = (uint64_t)x0 * y0;
    uint32_t h = 0;
    ZK_SHIFT(a, h, r0);
    col2(a, h, x0, y1, x1, y0);               ZK_SHIFT(a, h, r1);
    col3(a, h, x0, y2, x1, y1, x2, y0);       ZK_SHIFT(a, h, r2);
    col4(a, h, x0, y3, x1, y2, x2, y1, x3, y0); ZK_SHIFT(a, h, r3);
    col3(a, h, x1, y3, x2, y2, x3, y1);       ZK_SHIFT(a, h, r4);
    col2(a, h, x2, y3, x3, y2);               ZK_SHIFT(a, h, r5);
    col1(a, h, x3, y3);                       ZK_SHIFT(a, h, r6);
    r7 = (uint32_t)a;
}
#undef ZK_SHIFT

// ---- multiplication by a wave-uniform constant through its "W set" (DESIGN.md "What bounds the f128
// kernels").  For a constant w, W_i = w 2^(32i) mod p (i < 4), so a w = sum_i a_i W_i (mod p): a 162-bit sum
// of four 32 x 128-bit products, product-scanned in four columns, then ONE fold of its top 35 bits
// instead of the two folds of a 256-bit product.  29 % fewer issue slots than fe_mul (80 vs 113, tools/
// ubench/fmul_lab.hip).  The W words are read from SGPRs (scalar loads of a table the wave indexes
// uniformly), so the constant costs no VGPRs and no vector loads.
struct fe_ws {
    uint32_t w[16];  // w[4j + i] = 32-bit word j of W_i
};
__host__ inline fe_ws make_fe_ws(fe w);  // defined below the host fe_mul

// one column of the W-set product: like col3 / col4, the multiplier words in SGPRs
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

// (r0..r3) + (s4 + s5 2^32) 2^128 mod p for s5 < 2^3.  With T = s4 + s5 2^32 and S = L + T C:
// U = L - (T + 1) + ((T + 1) K) << 32 = S + C; the result is U - 2^128 when bit 128 of U is set (S >= p),
// else U - C (= S).  Carry chains with explicit SGPR pairs: 2 wait states between a VALU writing an SGPR
// and a VALU reading it (the s_nops); VALU -> SALU and SALU -> VALU need none here.
__device__ __forceinline__ fe ws_fold(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t s4, uint32_t s5) {
    const uint32_t K = 0x2d00u;
    const uint64_t m = (uint64_t)s4 * K + K;
    const uint32_t m0 = lo32(m), m1 = hi32(m) + s5 * K;
    uint32_t e0, e1, e2, e3, e4, u1, u2, u3, u4, nm, cw, o0, o1, o2, o3;
    uint64_t sB, sC, sD;
    const uint64_t ones = ~0ull;
    asm("v_subb_co_u32 %0, %15, %19, %23, %18\n\t"  // e0 = r0 - s4 - 1
        "s_nop 1\n\t"
        "v_subb_co_u32 %1, %15, %20, %24, %15\n\t"  // e1 = r1 - s5 - B
        "v_add_co_u32 %5, %16, %1, %25\n\t"         // u1 = e1 + m0
        "s_nop 0\n\t"
        "v_subb_co_u32 %2, %15, %21, 0, %15\n\t"    // e2
        "v_addc_co_u32 %6, %16, %2, %26, %16\n\t"   // u2 = e2 + m1 + c
        "s_nop 0\n\t"
        "v_subb_co_u32 %3, %15, %22, 0, %15\n\t"    // e3
        "v_addc_co_u32 %7, %16, %3, 0, %16\n\t"     // u3
        "s_nop 0\n\t"
        "v_subb_co_u32 %4, %15, 0, 0, %15\n\t"      // e4 = -B
        "v_addc_co_u32 %8, %16, %4, 0, %16\n\t"     // u4 = bit 128 of U
        "v_add_u32 %9, -1, %8\n\t"                  // nm: all ones when U < 2^128
        "v_and_b32 %10, 0x2cff, %9\n\t"
        "v_sub_co_u32 %11, %17, %0, %9\n\t"         // U - (nm ? C : 0)
        "s_nop 1\n\t"
        "v_subb_co_u32 %12, %17, %5, %10, %17\n\t"
        "s_nop 1\n\t"
        "v_subb_co_u32 %13, %17, %6, 0, %17\n\t"
        "s_nop 1\n\t"
        "v_subb_co_u32 %14, %17, %7, 0, %17"
        : "=&v"(e0), "=&v"(e1), "=&v"(e2), "=&v"(e3), "=&v"(e4), "=&v"(u1), "=&v"(u2), "=&v"(u3), "=&v"(u4), "=&v"(nm),
          "=&v"(cw), "=&v"(o0), "=&v"(o1), "=&v"(o2), "=&v"(o3), "=&s"(sB), "=&s"(sC), "=&s"(sD)
        : "s"(ones), "v"(r0), "v"(r1), "v"(r2), "v"(r3), "v"(s4), "v"(s5), "v"(m0), "v"(m1));
    return fe{join32(o0, o1), join32(o2, o3)};
}

// a * w for a wave-uniform constant w given by its W set (every word must be wave-uniform: load it with
// load_fe_ws at a uniform index)
__device__ __forceinline__ fe fe_mul_uniform(fe A, const fe_ws &W) {
    const uint32_t x0 = lo32(A.lo), x1 = hi32(A.lo), x2 = lo32(A.hi), x3 = hi32(A.hi);
    uint32_t r0, r1, r2, r3, h = 0;
    uint64_t a, kd;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(a), "=s"(kd) : "v"(x0), "s"(W.w[0]));
#define ZK_WSHIFT(out) do { out = (uint32_t)a; a = (a >> 32) | ((uint64_t)h << 32); h = 0; } while (0)
    col3s(a, h, x1, W.w[1], x2, W.w[2], x3, W.w[3]);                 ZK_WSHIFT(r0);
    col4s(a, h, x0, W.w[4], x1, W.w[5], x2, W.w[6], x3, W.w[7]);     ZK_WSHIFT(r1);
    col4s(a, h, x0, W.w[8], x1, W.w[9], x2, W.w[10], x3, W.w[11]);   ZK_WSHIFT(r2);
    col4s(a, h, x0, W.w[12], x1, W.w[13], x2, W.w[14], x3, W.w[15]); ZK_WSHIFT(r3);
#undef ZK_WSHIFT
    return ws_fold(r0, r1, r2, r3, (uint32_t)a, (uint32_t)(a >> 32));
}

// the same product with the W words in VGPRs: a W set shared by a group of lanes (vector loads), e.g. the NTT's
// group-uniform rounds (kernels.hip r4_round), where 16 lanes of a quarter-wave multiply by one twiddle
__device__ __forceinline__ void col3v(uint64_t &a, uint32_t &h, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                                      uint32_t x2, uint32_t y2) {
    uint64_t k0, k1, k2, kd;
    asm("v_mad_u64_u32 %0, %2, %6, %7, %0\n\t"
        "v_mad_u64_u32 %0, %3, %8, %9, %0\n\t"
        "v_mad_u64_u32 %0, %4, %10, %11, %0\n\t"
        "v_addc_co_u32 %1, %5, 0, 0, %2\n\t"
        "v_addc_co_u32 %1, %5, %1, 0, %3\n\t"
        "v_addc_co_u32 %1, %5, %1, 0, %4"
        : "+v"(a), "=&v"(h), "=&s"(k0), "=&s"(k1), "=&s"(k2), "=&s"(kd)
        : "v"(x0), "v"(y0), "v"(x1), "v"(y1), "v"(x2), "v"(y2));
}
__device__ __forceinline__ void col4v(uint64_t &a, uint32_t &h, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
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
        : "v"(x0), "v"(y0), "v"(x1), "v"(y1), "v"(x2), "v"(y2), "v"(x3), "v"(y3));
}
__device__ __forceinline__ fe fe_mul_wsv(fe A, const fe_ws &W) {
    const uint32_t x0 = lo32(A.lo), x1 = hi32(A.lo), x2 = lo32(A.hi), x3 = hi32(A.hi);
    uint32_t r0, r1, r2, r3, h = 0;
    uint64_t a = (uint64_t)x0 * W.w[0];
#define ZK_WSHIFT(out) do { out = (uint32_t)a; a = (a >> 32) | ((uint64_t)h << 32); h = 0; } while (0)
    col3v(a, h, x1, W.w[1], x2, W.w[2], x3, W.w[3]);                 ZK_WSHIFT(r0);
    col4v(a, h, x0, W.w[4], x1, W.w[5], x2, W.w[6], x3, W.w[7]);     ZK_WSHIFT(r1);
    col4v(a, h, x0, W.w[8], x1, W.w[9], x2, W.w[10], x3, W.w[11]);   ZK_WSHIFT(r2);
    col4v(a, h, x0, W.w[12], x1, W.w[13], x2, W.w[14], x3, W.w[15]); ZK_WSHIFT(r3);
#undef ZK_WSHIFT
    return ws_fold(r0, r1, r2, r3, (uint32_t)a, (uint32_t)(a >> 32));
}

// ---- two independent W-set products at once (the NTT butterflies multiply in pairs: x1 and x3 by one twiddle, a2 and
// a3 by two): the column products as above, then both final reductions in one list-scheduled asm block
// (addsub_asm.hpp ws_fold2_asm), whose two carry chains fill each other's wait states instead of s_nop.  ZK_FOLD2=0:
// two ws_folds, one after the other.  Same values.
#ifndef ZK_FOLD2
#define ZK_FOLD2 1
#endif
__device__ __forceinline__ void ws_fold2(uint32_t a[4], uint32_t as4, uint32_t as5, uint32_t b[4], uint32_t bs4,
                                         uint32_t bs5, fe &ra, fe &rb) {
    if constexpr (ZK_FOLD2) {
        const uint32_t K = 0x2d00u;
        const uint64_t ma = (uint64_t)as4 * K + K, mb = (uint64_t)bs4 * K + K;
        ws_fold2_asm(a, as4, as5, lo32(ma), hi32(ma) + as5 * K, b, bs4, bs5, lo32(mb), hi32(mb) + bs5 * K);
        ra = fe{join32(a[0], a[1]), join32(a[2], a[3])};
        rb = fe{join32(b[0], b[1]), join32(b[2], b[3])};
    } else {
        ra = ws_fold(a[0], a[1], a[2], a[3], as4, as5);
        rb = ws_fold(b[0], b[1], b[2], b[3], bs4, bs5);
    }
}
// the 160-bit column sums of A x W (W words from SGPRs): r[0..4) and the top (s4, s5)
__device__ __forceinline__ void ws_columns_s(fe A, const fe_ws &W, uint32_t r[4], uint32_t &s4, uint32_t &s5) {
    const uint32_t x0 = lo32(A.lo), x1 = hi32(A.lo), x2 = lo32(A.hi), x3 = hi32(A.hi);
    uint32_t h = 0;
    uint64_t a, kd;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(a), "=s"(kd) : "v"(x0), "s"(W.w[0]));
#define ZK_WSHIFT(out) do { out = (uint32_t)a; a = (a >> 32) | ((uint64_t)h << 32); h = 0; } while (0)
    col3s(a, h, x1, W.w[1], x2, W.w[2], x3, W.w[3]);                 ZK_WSHIFT(r[0]);
    col4s(a, h, x0, W.w[4], x1, W.w[5], x2, W.w[6], x3, W.w[7]);     ZK_WSHIFT(r[1]);
    col4s(a, h, x0, W.w[8], x1, W.w[9], x2, W.w[10], x3, W.w[11]);   ZK_WSHIFT(r[2]);
    col4s(a, h, x0, W.w[12], x1, W.w[13], x2, W.w[14], x3, W.w[15]); ZK_WSHIFT(r[3]);
#undef ZK_WSHIFT
    s4 = (uint32_t)a;
    s5 = (uint32_t)(a >> 32);
}
// ... the W words in VGPRs (a W set shared by a group of lanes)
__device__ __forceinline__ void ws_columns_v(fe A, const fe_ws &W, uint32_t r[4], uint32_t &s4, uint32_t &s5) {
    const uint32_t x0 = lo32(A.lo), x1 = hi32(A.lo), x2 = lo32(A.hi), x3 = hi32(A.hi);
    uint32_t h = 0;
    uint64_t a = (uint64_t)x0 * W.w[0];
#define ZK_WSHIFT(out) do { out = (uint32_t)a; a = (a >> 32) | ((uint64_t)h << 32); h = 0; } while (0)
    col3v(a, h, x1, W.w[1], x2, W.w[2], x3, W.w[3]);                 ZK_WSHIFT(r[0]);
    col4v(a, h, x0, W.w[4], x1, W.w[5], x2, W.w[6], x3, W.w[7]);     ZK_WSHIFT(r[1]);
    col4v(a, h, x0, W.w[8], x1, W.w[9], x2, W.w[10], x3, W.w[11]);   ZK_WSHIFT(r[2]);
    col4v(a, h, x0, W.w[12], x1, W.w[13], x2, W.w[14], x3, W.w[15]); ZK_WSHIFT(r[3]);
#undef ZK_WSHIFT
    s4 = (uint32_t)a;
    s5 = (uint32_t)(a >> 32);
}
// ra = A * WA, rb = B * WB (wave-uniform W sets, scalar loads)
__device__ __forceinline__ void fe_mul_uniform2(fe A, const fe_ws &WA, fe B, const fe_ws &WB, fe &ra, fe &rb) {
    uint32_t a[4], b[4], as4, as5, bs4, bs5;
    ws_columns_s(A, WA, a, as4, as5);
    ws_columns_s(B, WB, b, bs4, bs5);
    ws_fold2(a, as4, as5, b, bs4, bs5, ra, rb);
}
// ... group-uniform W sets (vector loads)
__device__ __forceinline__ void fe_mul_wsv2(fe A, const fe_ws &WA, fe B, const fe_ws &WB, fe &ra, fe &rb) {
    uint32_t a[4], b[4], as4, as5, bs4, bs5;
    ws_columns_v(A, WA, a, as4, as5);
    ws_columns_v(B, WB, b, bs4, bs5);
    ws_fold2(a, as4, as5, b, bs4, bs5, ra, rb);
}

// The pair forms where the kernel's register budget has room for them (F2: kernels.hip chooses per call site), else
// the two products one after the other.  Same values.
template <bool F2>
__device__ __forceinline__ void mul_uniform_pair(fe A, const fe_ws &WA, fe B, const fe_ws &WB, fe &ra, fe &rb) {
    if constexpr (F2) {
        fe_mul_uniform2(A, WA, B, WB, ra, rb);
    } else {
        ra = fe_mul_uniform(A, WA);
        rb = fe_mul_uniform(B, WB);
    }
}
template <bool F2>
__device__ __forceinline__ void mul_wsv_pair(fe A, const fe_ws &WA, fe B, const fe_ws &WB, fe &ra, fe &rb) {
    if constexpr (F2) {
        fe_mul_wsv2(A, WA, B, WB, ra, rb);
    } else {
        ra = fe_mul_wsv(A, WA);
        rb = fe_mul_wsv(B, WB);
    }
}

// ---- per-lane constant in two parts (32 B): a w = (a mod 2^64) w + (a >> 64) (w 2^64 mod p), a 193-bit sum
// of two 64 x 128-bit products (five columns), one K-fold of its top 65 bits (H C = H K 2^32 - H), then
// ws_fold's final step.  99 issue slots against fe_mul's 113 (tools/ubench/fmul_lab.hip v5): for per-lane
// twiddles, where a 64-B W set per lane costs more in loads than it saves.
struct fe_w2 {
    fe w, w64;  // w and w 2^64 mod p
};
__device__ __forceinline__ fe fe_mul_w2(fe A, const fe_w2 &W) {
    const uint32_t x0 = lo32(A.lo), x1 = hi32(A.lo), x2 = lo32(A.hi), x3 = hi32(A.hi);
    const uint32_t a0 = lo32(W.w.lo), a1 = hi32(W.w.lo), a2 = lo32(W.w.hi), a3 = hi32(W.w.hi);
    const uint32_t b0 = lo32(W.w64.lo), b1 = hi32(W.w64.lo), b2 = lo32(W.w64.hi), b3 = hi32(W.w64.hi);
    uint32_t r0, r1, r2, r3, r4, h = 0;
    uint64_t a = (uint64_t)x0 * a0;
#define ZK_WSHIFT(out) do { out = (uint32_t)a; a = (a >> 32) | ((uint64_t)h << 32); h = 0; } while (0)
    col1(a, h, x2, b0);                          ZK_WSHIFT(r0);
    col4(a, h, x0, a1, x1, a0, x2, b1, x3, b0);  ZK_WSHIFT(r1);
    col4(a, h, x0, a2, x1, a1, x2, b2, x3, b1);  ZK_WSHIFT(r2);
    col4(a, h, x0, a3, x1, a2, x2, b3, x3, b2);  ZK_WSHIFT(r3);
    col2(a, h, x1, a3, x3, b3);                  ZK_WSHIFT(r4);
#undef ZK_WSHIFT
    const uint32_t s5 = (uint32_t)a, s6 = (uint32_t)(a >> 32);  // s6 <= 1
    // S' = L - H + (H K) << 32 with H = r4 + s5 2^32 + s6 2^64; S' < 2^128 + 2^111, bit 128 in e4
    const uint32_t K = 0x2d00u;
    uint64_t q = (uint64_t)r4 * K;
    const uint32_t q0 = lo32(q);
    q = (uint64_t)s5 * K + (q >> 32);
    const uint32_t q1 = lo32(q), q2 = hi32(q) + s6 * K;
    uint32_t d0, d1, d2, d3, dm, e1, e2, e3, e4;
    uint64_t sB, sC;
    asm("v_sub_co_u32 %0, %9, %11, %15\n\t"        // d0 = r0 - r4
        "s_nop 1\n\t"
        "v_subb_co_u32 %1, %9, %12, %16, %9\n\t"   // d1 = r1 - s5 - b
        "v_add_co_u32 %5, %10, %1, %18\n\t"        // e1 = d1 + q0
        "s_nop 0\n\t"
        "v_subb_co_u32 %2, %9, %13, %17, %9\n\t"   // d2 = r2 - s6 - b
        "v_addc_co_u32 %6, %10, %2, %19, %10\n\t"  // e2 = d2 + q1 + c
        "s_nop 0\n\t"
        "v_subb_co_u32 %3, %9, %14, 0, %9\n\t"     // d3
        "v_addc_co_u32 %7, %10, %3, %20, %10\n\t"  // e3 = d3 + q2 + c
        "s_nop 0\n\t"
        "v_subb_co_u32 %4, %9, 0, 0, %9\n\t"       // dm = -b
        "v_addc_co_u32 %8, %10, %4, 0, %10"        // e4
        : "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "=&v"(dm), "=&v"(e1), "=&v"(e2), "=&v"(e3), "=&v"(e4), "=&s"(sB),
          "=&s"(sC)
        : "v"(r0), "v"(r1), "v"(r2), "v"(r3), "v"(r4), "v"(s5), "v"(s6), "v"(q0), "v"(q1), "v"(q2));
    return ws_fold(d0, e1, e2, e3, e4, 0u);
}
// two per-lane two-part products (fe_mul_w2) with their final reductions paired (ws_fold2)
__device__ __forceinline__ void w2_head(fe A, const fe_w2 &W, uint32_t o[4], uint32_t &o4) {
    const uint32_t x0 = lo32(A.lo), x1 = hi32(A.lo), x2 = lo32(A.hi), x3 = hi32(A.hi);
    const uint32_t a0 = lo32(W.w.lo), a1 = hi32(W.w.lo), a2 = lo32(W.w.hi), a3 = hi32(W.w.hi);
    const uint32_t b0 = lo32(W.w64.lo), b1 = hi32(W.w64.lo), b2 = lo32(W.w64.hi), b3 = hi32(W.w64.hi);
    uint32_t r0, r1, r2, r3, r4, h = 0;
    uint64_t a = (uint64_t)x0 * a0;
#define ZK_WSHIFT(out) do { out = (uint32_t)a; a = (a >> 32) | ((uint64_t)h << 32); h = 0; } while (0)
    col1(a, h, x2, b0);                          ZK_WSHIFT(r0);
    col4(a, h, x0, a1, x1, a0, x2, b1, x3, b0);  ZK_WSHIFT(r1);
    col4(a, h, x0, a2, x1, a1, x2, b2, x3, b1);  ZK_WSHIFT(r2);
    col4(a, h, x0, a3, x1, a2, x2, b3, x3, b2);  ZK_WSHIFT(r3);
    col2(a, h, x1, a3, x3, b3);                  ZK_WSHIFT(r4);
#undef ZK_WSHIFT
    const uint32_t s5 = (uint32_t)a, s6 = (uint32_t)(a >> 32);
    const uint32_t K = 0x2d00u;
    uint64_t q = (uint64_t)r4 * K;
    const uint32_t q0 = lo32(q);
    q = (uint64_t)s5 * K + (q >> 32);
    const uint32_t q1 = lo32(q), q2 = hi32(q) + s6 * K;
    uint32_t d1, d2, d3, dm;
    uint64_t sB, sC;
    asm("v_sub_co_u32 %0, %9, %11, %15\n\t"
        "s_nop 1\n\t"
        "v_subb_co_u32 %1, %9, %12, %16, %9\n\t"
        "v_add_co_u32 %5, %10, %1, %18\n\t"
        "s_nop 0\n\t"
        "v_subb_co_u32 %2, %9, %13, %17, %9\n\t"
        "v_addc_co_u32 %6, %10, %2, %19, %10\n\t"
        "s_nop 0\n\t"
        "v_subb_co_u32 %3, %9, %14, 0, %9\n\t"
        "v_addc_co_u32 %7, %10, %3, %20, %10\n\t"
        "s_nop 0\n\t"
        "v_subb_co_u32 %4, %9, 0, 0, %9\n\t"
        "v_addc_co_u32 %8, %10, %4, 0, %10"
        : "=&v"(o[0]), "=&v"(d1), "=&v"(d2), "=&v"(d3), "=&v"(dm), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o4),
          "=&s"(sB), "=&s"(sC)
        : "v"(r0), "v"(r1), "v"(r2), "v"(r3), "v"(r4), "v"(s5), "v"(s6), "v"(q0), "v"(q1), "v"(q2));
}
__device__ __forceinline__ void fe_mul_w2_2(fe A, const fe_w2 &WA, fe B, const fe_w2 &WB, fe &ra, fe &rb) {
    uint32_t a[4], b[4], a4, b4;
    w2_head(A, WA, a, a4);
    w2_head(B, WB, b, b4);
    ws_fold2(a, a4, 0u, b, b4, 0u, ra, rb);
}
template <bool F2>
__device__ __forceinline__ void mul_w2_pair(fe A, const fe_w2 &WA, fe B, const fe_w2 &WB, fe &ra, fe &rb) {
    if constexpr (F2) {
        fe_mul_w2_2(A, WA, B, WB, ra, rb);
    } else {
        ra = fe_mul_w2(A, WA);
        rb = fe_mul_w2(B, WB);
    }
}

// ---- two butterflies' sums and differences at once: (a + b, a - b, c + d, c - d) mod p.  ZK_ADDSUB_ASM (default):
// the four carry chains as one list-scheduled asm block on their own SGPR pairs (addsub_asm.hpp, generated by
// tools/gen_addsub_asm.py), so the wait states between a carry write and its read are filled by the other chains
// instead of s_nop, and each difference takes one lane-mask select instead of two; otherwise the compiler's
// chains through VCC, one after the other.  Same values either way.
#ifndef ZK_ADDSUB_ASM
#define ZK_ADDSUB_ASM 1
#endif
// V: 0 both sums canonical, 1 both lazy (fe_add_lazy's contract: a, c any value < 2^128; b, d canonical),
// 2 the first lazy and the second canonical
template <int V>
__device__ __forceinline__ void addsub2_v(fe a, fe b, fe c, fe d, fe &apb, fe &amb, fe &cpd, fe &cmd) {
    if constexpr (ZK_ADDSUB_ASM) {
        uint32_t A[4] = {lo32(a.lo), hi32(a.lo), lo32(a.hi), hi32(a.hi)};
        uint32_t B[4] = {lo32(b.lo), hi32(b.lo), lo32(b.hi), hi32(b.hi)};
        uint32_t C[4] = {lo32(c.lo), hi32(c.lo), lo32(c.hi), hi32(c.hi)};
        uint32_t D[4] = {lo32(d.lo), hi32(d.lo), lo32(d.hi), hi32(d.hi)};
        uint32_t S[4], E[4];
        if constexpr (V == 0) addsub2_asm_cc(A, B, C, D, S, E);
        else if constexpr (V == 1) addsub2_asm_ll(A, B, C, D, S, E);
        else addsub2_asm_lc(A, B, C, D, S, E);
        apb = fe{join32(A[0], A[1]), join32(A[2], A[3])};
        amb = fe{join32(S[0], S[1]), join32(S[2], S[3])};
        cpd = fe{join32(C[0], C[1]), join32(C[2], C[3])};
        cmd = fe{join32(E[0], E[1]), join32(E[2], E[3])};
    } else {
        apb = V != 0 ? fe_add_lazy(a, b) : fe_add(a, b);
        amb = fe_sub(a, b);
        cpd = V == 1 ? fe_add_lazy(c, d) : fe_add(c, d);
        cmd = fe_sub(c, d);
    }
}
__device__ __forceinline__ void fe_addsub2(fe a, fe b, fe c, fe d, fe &apb, fe &amb, fe &cpd, fe &cmd) {
    addsub2_v<0>(a, b, c, d, apb, amb, cpd, cmd);
}
// the same with lazy sums (fe_add_lazy's contract: a, c any value < 2^128; b, d canonical)
template <bool LZ>
__device__ __forceinline__ void addsub2(fe a, fe b, fe c, fe d, fe &apb, fe &amb, fe &cpd, fe &cmd) {
    addsub2_v<LZ ? 1 : 0>(a, b, c, d, apb, amb, cpd, cmd);
}

// the W set tab[idx] for a wave-uniform idx, through scalar loads
__device__ __forceinline__ fe_ws load_fe_ws(const fe_ws *__restrict__ tab, int idx) {
    fe_ws r;
    idx = __builtin_amdgcn_readfirstlane(idx);
#pragma unroll
    for (int k = 0; k < 16; k++) r.w[k] = __builtin_amdgcn_readfirstlane(tab[idx].w[k]);
    return r;
}

__device__ __forceinline__ fe fe_mul_asm(fe A, fe Bv) {
    uint32_t r[8];
    mul_wide(A, Bv, r);
    return reduce_fold(r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
}
__host__ inline void mul_wide(fe a, fe b, uint32_t r[8]) {
    const uint32_t x[4] = {lo32(a.lo), hi32(a.lo), lo32(a.hi), hi32(a.hi)};
    const uint32_t y[4] = {lo32(b.lo), hi32(b.lo), lo32(b.hi), hi32(b.hi)};
    mul_4x4(x, y, r);
}

// Lazy dot products: sum unreduced 256-bit products in 288 bits (up to 2^32 terms) and reduce once.
// 2^256 = C^2 (mod p) with C^2 < 2^92 < p, so the top limb folds in as w8 * C^2 < 2^124.
struct acc288 {
    uint32_t w[9];
};
ZK_HD acc288 acc288_zero() { return acc288{{0, 0, 0, 0, 0, 0, 0, 0, 0}}; }
ZK_HD void acc288_madd(acc288 &acc, fe a, fe b) {
    uint32_t r[8], c;
#ifdef __HIP_DEVICE_COMPILE__
    // order the products by the accumulation chain: an unreduced product holds 8 VGPRs, and left
    // alone the scheduler computes every product of a long sum up front
    asm volatile("" : "+v"(a.lo), "+v"(a.hi) : "v"(acc.w[0]));
#endif
    mul_wide(a, b, r);
    acc.w[0] = __builtin_addc(acc.w[0], r[0], 0u, &c);
#pragma unroll
    for (int k = 1; k < 8; k++) acc.w[k] = __builtin_addc(acc.w[k], r[k], c, &c);
    acc.w[8] += c;
}
ZK_HD fe acc288_reduce(const acc288 &acc) {
    const fe v = reduce_fold(acc.w[0], acc.w[1], acc.w[2], acc.w[3], acc.w[4], acc.w[5], acc.w[6], acc.w[7]);
    // w8 * C^2 with C^2 = 2025*2^80 - 90*2^40 + 1 (92 bits), as (lo 64, hi 28) limbs
    constexpr uint64_t C2_LO = (uint64_t)(((unsigned __int128)ZK_C * ZK_C) & ~0ULL);
    constexpr uint64_t C2_HI = (uint64_t)(((unsigned __int128)ZK_C * ZK_C) >> 64);
    const uint64_t t_lo = (uint64_t)lo32(C2_LO) * acc.w[8];
    const uint64_t t_mid = (uint64_t)hi32(C2_LO) * acc.w[8] + (t_lo >> 32);
    const uint64_t t_hi = C2_HI * acc.w[8] + (t_mid >> 32);  // < 2^60
    const fe top = fe{(t_lo & 0xffffffffull) | (t_mid << 32), t_hi};
    return fe_add(v, top);
}

// device and host overloads (clang resolves by target)
__device__ __forceinline__ fe fe_mul(fe a, fe b) { return fe_mul_asm(a, b); }
// host: unsigned __int128 with the same two folds
__host__ static inline fe fe_from_u128(unsigned __int128 v) { return fe{(uint64_t)v, (uint64_t)(v >> 64)}; }
__host__ static inline unsigned __int128 fe_to_u128(fe a) { return ((unsigned __int128)a.hi << 64) | a.lo; }
// hi * 2^128 + lo (mod p) for any 256-bit value
__host__ static inline fe fe_reduce_wide(unsigned __int128 lo, unsigned __int128 hi) {
    typedef unsigned __int128 u128;
    const u128 P = ((u128)ZK_P_HI << 64) | ZK_P_LO;
    // 2^128 = C (mod p), C < 2^46: lo + hi*C = s2 + top * 2^128 with top < 2^47, then fold once more
    const u128 t0 = (u128)(uint64_t)hi * ZK_C, t1 = (u128)(uint64_t)(hi >> 64) * ZK_C;
    const u128 s1 = lo + t0;
    const u128 s2 = s1 + (t1 << 64);
    const uint64_t top = (uint64_t)(t1 >> 64) + (uint64_t)(s1 < lo) + (uint64_t)(s2 < s1);
    u128 r = s2 + (u128)top * ZK_C;
    if (r < s2) r += ZK_C;  // wrapped past 2^128: + 2^128 = + C (mod p); cannot wrap again
    if (r >= P) r -= P;
    return fe_from_u128(r);
}
__host__ static inline fe fe_mul(fe a, fe b) {
    typedef unsigned __int128 u128;
    const u128 p00 = (u128)a.lo * b.lo, p01 = (u128)a.lo * b.hi, p10 = (u128)a.hi * b.lo, p11 = (u128)a.hi * b.hi;
    const u128 mid = (p00 >> 64) + (uint64_t)p01 + (uint64_t)p10;
    const u128 lo = (mid << 64) | (uint64_t)p00;
    const u128 hi = p11 + (p01 >> 64) + (p10 >> 64) + (mid >> 64);  // product = hi * 2^128 + lo
    return fe_reduce_wide(lo, hi);
}
// a^2 with three 64 x 64 products (the cross product once, doubled)
__host__ static inline fe fe_sqr_host(fe a) {
    typedef unsigned __int128 u128;
    const u128 p00 = (u128)a.lo * a.lo, p01 = (u128)a.lo * a.hi, p11 = (u128)a.hi * a.hi;
    const u128 mid = (p00 >> 64) + (u128)(uint64_t)p01 * 2;  // < 3 * 2^64
    const u128 lo = (mid << 64) | (uint64_t)p00;
    const u128 hi = p11 + (p01 >> 64) * 2 + (mid >> 64);
    return fe_reduce_wide(lo, hi);
}

ZK_HD fe fe_sqr(fe a) { return fe_mul(a, a); }

__host__ inline fe_w2 make_fe_w2(fe w) {
    const fe two64 = fe{0, 1};
    return fe_w2{w, fe_mul(w, two64)};
}
__host__ inline fe_ws make_fe_ws(fe w) {
    fe_ws W;
    const fe two32 = fe{1ull << 32, 0};
    for (int i = 0; i < 4; i++) {
        W.w[0 + i] = lo32(w.lo);
        W.w[4 + i] = hi32(w.lo);
        W.w[8 + i] = lo32(w.hi);
        W.w[12 + i] = hi32(w.hi);
        w = fe_mul(w, two32);
    }
    return W;
}

// ---- multiply-accumulate by small (< 2^32) constants, reduced once: for the Rescue MDS matrix,
// whose entries are small signed integers (crypto/src/rescue.rs:197-214).
struct acc160 {
    uint32_t w[5];
};
ZK_HD acc160 acc160_zero() { return acc160{{0, 0, 0, 0, 0}}; }
// acc += x * c  (acc stays < 2^160 for a handful of terms)
ZK_HD void acc160_madd(acc160 &acc, fe x, uint32_t c) {
    const uint32_t xs[4] = {lo32(x.lo), hi32(x.lo), lo32(x.hi), hi32(x.hi)};
    uint64_t t = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        t = (uint64_t)xs[k] * c + acc.w[k] + (t >> 32);
        acc.w[k] = lo32(t);
    }
    acc.w[4] += hi32(t);
}
// reduce a < 2^160 value: L + H*C with H < 2^32, C = 45*2^40 - 1
ZK_HD fe acc160_reduce(const acc160 &a) {
    uint64_t lo = (uint64_t)a.w[0] | ((uint64_t)a.w[1] << 32);
    uint64_t hi = (uint64_t)a.w[2] | ((uint64_t)a.w[3] << 32);
    uint64_t sh = a.w[4];
    uint64_t q = sh * 45u;
    uint64_t add_lo = q << 40, add_hi = q >> 24;
    uint64_t nlo = lo + add_lo;
    uint64_t c = nlo < lo;
    uint64_t nhi = hi + add_hi + c;
    uint64_t carry = (nhi < hi) | ((nhi == hi) & c);
    uint64_t blo = nlo - sh;
    uint64_t b = nlo < sh;
    uint64_t bhi = nhi - b;
    carry -= (nhi < b);
    uint64_t clo = blo + (carry ? ZK_C : 0);
    uint64_t chi = bhi + (clo < blo);
    uint64_t ulo = clo + ZK_C;
    uint64_t uhi = chi + (ulo < clo);
    bool ge = uhi < chi;
    return fe{ge ? ulo : clo, ge ? uhi : chi};
}

ZK_HD fe fe_exp(fe b, uint64_t e_lo, uint64_t e_hi = 0) {
    // right-to-left square and multiply over the 128-bit exponent (e_hi:e_lo)
    fe r = fe_one();
    for (int i = 0; i < 128; i++) {
        uint64_t word = i < 64 ? e_lo : e_hi;
        int sh = i & 63;
        uint64_t remaining = (word >> sh) | (i < 64 ? e_hi : 0);
        if (remaining == 0) break;
        if ((word >> sh) & 1) r = fe_mul(r, b);
        b = fe_mul(b, b);
    }
    return r;
}

// a^(2^k) by repeated squaring
ZK_HD fe fe_sqr_n(fe a, int k) {
    for (int i = 0; i < k; i++) a = fe_mul(a, a);
    return a;
}

// a^(p-2) with an addition chain: p-2 = 0xffffffffffffffff_ffffd2ff_ffffffff
// = (2^80 - 1) * 2^48 + 0xd2 * 2^40 + (2^40 - 1).   143 multiplications in total.
ZK_HD fe fe_inv(fe a) {
    fe x1 = a;
    fe x2 = fe_mul(fe_sqr_n(x1, 1), x1);
    fe x4 = fe_mul(fe_sqr_n(x2, 2), x2);
    fe x8 = fe_mul(fe_sqr_n(x4, 4), x4);
    fe x16 = fe_mul(fe_sqr_n(x8, 8), x8);
    fe x32 = fe_mul(fe_sqr_n(x16, 16), x16);
    fe x40 = fe_mul(fe_sqr_n(x32, 8), x8);
    fe x80 = fe_mul(fe_sqr_n(x40, 40), x40);  // a^(2^80 - 1)
    // append the byte 0xd2 = 1101 0010
    fe r = x80;
    const int bits[8] = {1, 1, 0, 1, 0, 0, 1, 0};
    for (int i = 0; i < 8; i++) {
        r = fe_mul(r, r);
        if (bits[i]) r = fe_mul(r, a);
    }
    // append 40 ones
    r = fe_mul(fe_sqr_n(r, 40), x40);
    return r;
}

ZK_HD fe fe_from_u64(uint64_t v) { return fe{v, 0}; }
