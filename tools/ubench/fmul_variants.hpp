// candidate device multiplies for tools/ubench/fmul_lab.hip (variant 0 = the library's fe_mul)
#pragma once
#define FMUL_NVARIANTS 6
static const char *fmul_variant_name(int v) {
    static const char *n[] = {"library fe_mul", "v1: U = T + C final step", "v2: independent fold products, mask final step",
                              "v3: precomputed W_i = b 2^(32i) mod p (16 words), one 35-bit fold",
                              "v4: as v3, two products sharing one W set",
                              "v5: two constants w, w 2^64 mod p (per-lane form, 32 B)"};
    return n[v];
}

__device__ __forceinline__ fe reduce_v1(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t r4, uint32_t r5,
                                        uint32_t r6, uint32_t r7) {
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
    const uint32_t dm = 0u - b;
    const uint32_t s1 = __builtin_addc(d1, q0, 0u, &c);
    const uint32_t s2 = __builtin_addc(d2, q1, c, &c);
    const uint32_t s3 = __builtin_addc(d3, q2, c, &c);
    const uint32_t s4 = __builtin_addc(dm, q3, c, &c);
    const uint32_t s5 = dm + q4 + c;
    uint64_t m = (uint64_t)s4 * K + K;
    const uint32_t m0 = lo32(m);
    m = (uint64_t)s5 * K + (m >> 32);
    const uint32_t m1 = lo32(m);
    uint32_t B, Cy;
    const uint32_t e0 = __builtin_subc(d0, s4, 1u, &B);
    const uint32_t e1 = __builtin_subc(s1, s5, B, &B);
    const uint32_t e2 = __builtin_subc(s2, 0u, B, &B);
    const uint32_t e3 = __builtin_subc(s3, 0u, B, &B);
    const uint32_t u1 = __builtin_addc(e1, m0, 0u, &Cy);
    const uint32_t u2 = __builtin_addc(e2, m1, Cy, &Cy);
    const uint32_t u3 = __builtin_addc(e3, 0u, Cy, &Cy);
    const bool hi = Cy && !B;
    const uint32_t cw0 = hi ? 0u : 0xffffffffu, cw1 = hi ? 0u : 0x2cffu;
    uint32_t bb;
    const uint32_t o0 = __builtin_subc(e0, cw0, 0u, &bb);
    const uint32_t o1 = __builtin_subc(u1, cw1, bb, &bb);
    const uint32_t o2 = __builtin_subc(u2, 0u, bb, &bb);
    const uint32_t o3 = __builtin_subc(u3, 0u, bb, &bb);
    return fe{join32(o0, o1), join32(o2, o3)};
}
__device__ __forceinline__ fe reduce_v2(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t r4, uint32_t r5,
                                        uint32_t r6, uint32_t r7) {
    const uint32_t K = 0x2d00u;
    const uint64_t P0 = (uint64_t)r4 * K, P1 = (uint64_t)r5 * K, P2 = (uint64_t)r6 * K, P3 = (uint64_t)r7 * K;
    uint32_t b, c;
    const uint32_t d0 = __builtin_subc(r0, r4, 0u, &b);
    const uint32_t d1 = __builtin_subc(r1, r5, b, &b);
    const uint32_t d2 = __builtin_subc(r2, r6, b, &b);
    const uint32_t d3 = __builtin_subc(r3, r7, b, &b);
    const uint32_t dm = __builtin_subc(0u, 0u, b, &b);  // -borrow
    uint32_t s1 = __builtin_addc(d1, lo32(P0), 0u, &c);
    uint32_t s2 = __builtin_addc(d2, lo32(P1), c, &c);
    uint32_t s3 = __builtin_addc(d3, lo32(P2), c, &c);
    uint32_t s4 = __builtin_addc(dm, lo32(P3), c, &c);
    uint32_t s5 = dm + c;
    s2 = __builtin_addc(s2, hi32(P0), 0u, &c);
    s3 = __builtin_addc(s3, hi32(P1), c, &c);
    s4 = __builtin_addc(s4, hi32(P2), c, &c);
    s5 = s5 + hi32(P3) + c;
    // U = S_lo - S_hi - 1 + ((S_hi + 1) * K) << 32: (S_hi + 1) K = M0 + M1 << 32, M1 = s5 K < 2^29
    const uint64_t M0 = (uint64_t)s4 * K + K;
    const uint32_t w1 = hi32(M0) + s5 * K;
    uint32_t B, Cy;
    const uint32_t e0 = __builtin_subc(d0, s4 + 1u, 0u, &B);  // s4 + 1 wraps only when s4 = 2^32 - 1
    const uint32_t e1 = __builtin_subc(s1, s5 + (s4 == 0xffffffffu), B, &B);
    const uint32_t e2 = __builtin_subc(s2, 0u, B, &B);
    const uint32_t e3 = __builtin_subc(s3, 0u, B, &B);
    const uint32_t e4 = __builtin_subc(0u, 0u, B, &B);
    const uint32_t u1 = __builtin_addc(e1, lo32(M0), 0u, &Cy);
    const uint32_t u2 = __builtin_addc(e2, w1, Cy, &Cy);
    const uint32_t u3 = __builtin_addc(e3, 0u, Cy, &Cy);
    const uint32_t u4 = e4 + Cy;            // bit 128 of U (0 or 1)
    const uint32_t nm = u4 - 1u;            // all ones when U < 2^128: subtract C
    uint32_t bb;
    const uint32_t o0 = __builtin_subc(e0, nm, 0u, &bb);
    const uint32_t o1 = __builtin_subc(u1, nm & 0x2cffu, bb, &bb);
    const uint32_t o2 = __builtin_subc(u2, 0u, bb, &bb);
    const uint32_t o3 = __builtin_subc(u3, 0u, bb, &bb);
    return fe{join32(o0, o1), join32(o2, o3)};
}


// ---- multiply by a precomputed constant: x * w = sum_i x_i (w 2^(32i) mod p) (mod p).  Wc[4j + i] is
// word j of W_i = w 2^(32i) mod p.  The four columns of the 162-bit sum are product-scanned (4 MADs each),
// the top 35 bits T = s4 + s5 2^32 fold once: U = L - (T + 1) + ((T + 1) K) << 32 = S + C, and the result
// is U - 2^128 when bit 128 of U is set, else U - C.
struct WSet {
    uint32_t w[16];
};
__host__ inline WSet make_wset(fe b) {
    WSet W;
    fe t = b;
    const fe two32 = fe{1ull << 32, 0};
    for (int i = 0; i < 4; i++) {
        W.w[0 * 4 + i] = lo32(t.lo);
        W.w[1 * 4 + i] = hi32(t.lo);
        W.w[2 * 4 + i] = lo32(t.hi);
        W.w[3 * 4 + i] = hi32(t.hi);
        t = fe_mul(t, two32);
    }
    return W;
}
#define ZK_SHIFT2(a, h, out) do { out = (uint32_t)(a); a = ((a) >> 32) | ((uint64_t)(h) << 32); h = 0; } while (0)
__device__ __forceinline__ void pre_cols(fe A, const uint32_t *W, uint32_t &r0, uint32_t &r1, uint32_t &r2, uint32_t &r3,
                                         uint32_t &s4, uint32_t &s5) {
    const uint32_t x0 = lo32(A.lo), x1 = hi32(A.lo), x2 = lo32(A.hi), x3 = hi32(A.hi);
    uint64_t a = (uint64_t)x0 * W[0];
    uint32_t h = 0;
    col3(a, h, x1, W[1], x2, W[2], x3, W[3]);               ZK_SHIFT2(a, h, r0);
    col4(a, h, x0, W[4], x1, W[5], x2, W[6], x3, W[7]);     ZK_SHIFT2(a, h, r1);
    col4(a, h, x0, W[8], x1, W[9], x2, W[10], x3, W[11]);   ZK_SHIFT2(a, h, r2);
    col4(a, h, x0, W[12], x1, W[13], x2, W[14], x3, W[15]); ZK_SHIFT2(a, h, r3);
    s4 = (uint32_t)a;
    s5 = (uint32_t)(a >> 32);
}
// fold of (r0..r3) + (s4 + s5 2^32) 2^128, s5 < 8; hazard rule: 2 wait states between a VALU SGPR write
// and a VALU read of it
__device__ __forceinline__ fe pre_fold(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t s4, uint32_t s5) {
    const uint32_t K = 0x2d00u;
    const uint64_t m = (uint64_t)s4 * K + K;
    const uint32_t m0 = lo32(m), m1 = hi32(m) + s5 * K;
    uint32_t e0, e1, e2, e3, e4, u1, u2, u3, u4, nm, cw, o0, o1, o2, o3;
    uint64_t sB, sC, sD;
    const uint64_t ones = ~0ull;
    asm("v_subb_co_u32 %0, %15, %19, %23, %18\n\t"   // e0 = r0 - s4 - 1
        "s_nop 1\n\t"
        "v_subb_co_u32 %1, %15, %20, %24, %15\n\t"   // e1 = r1 - s5 - B
        "v_add_co_u32 %5, %16, %1, %25\n\t"          // u1 = e1 + m0
        "s_nop 0\n\t"
        "v_subb_co_u32 %2, %15, %21, 0, %15\n\t"     // e2
        "v_addc_co_u32 %6, %16, %2, %26, %16\n\t"    // u2 = e2 + m1 + c
        "s_nop 0\n\t"
        "v_subb_co_u32 %3, %15, %22, 0, %15\n\t"     // e3
        "v_addc_co_u32 %7, %16, %3, 0, %16\n\t"      // u3
        "s_nop 0\n\t"
        "v_subb_co_u32 %4, %15, 0, 0, %15\n\t"       // e4 = -B
        "v_addc_co_u32 %8, %16, %4, 0, %16\n\t"      // u4 = bit 128 of U
        "v_add_u32 %9, -1, %8\n\t"                   // nm: all ones when U < 2^128
        "v_and_b32 %10, 0x2cff, %9\n\t"
        "v_sub_co_u32 %11, %17, %0, %9\n\t"          // U - (nm ? C : 0)
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
__device__ __forceinline__ fe fe_mul_pre(fe a, const uint32_t *W) {
    uint32_t r0, r1, r2, r3, s4, s5;
    pre_cols(a, W, r0, r1, r2, r3, s4, s5);
    return pre_fold(r0, r1, r2, r3, s4, s5);
}

// ---- per-lane constant in two parts: a w = (a mod 2^64) w + (a >> 64) (w 2^64 mod p), a 193-bit sum of two
// 64 x 128-bit products (five columns), one K-fold of its top 65 bits, then ws_fold's final step.
__device__ __forceinline__ fe fe_mul_w2(fe A, fe W0, fe W2) {
    const uint32_t x0 = lo32(A.lo), x1 = hi32(A.lo), x2 = lo32(A.hi), x3 = hi32(A.hi);
    const uint32_t a0 = lo32(W0.lo), a1 = hi32(W0.lo), a2 = lo32(W0.hi), a3 = hi32(W0.hi);
    const uint32_t b0 = lo32(W2.lo), b1 = hi32(W2.lo), b2 = lo32(W2.hi), b3 = hi32(W2.hi);
    uint32_t r0, r1, r2, r3, r4;
    uint64_t a = (uint64_t)x0 * a0;
    uint32_t h = 0;
    col1(a, h, x2, b0);                                   ZK_SHIFT2(a, h, r0);
    col4(a, h, x0, a1, x1, a0, x2, b1, x3, b0);           ZK_SHIFT2(a, h, r1);
    col4(a, h, x0, a2, x1, a1, x2, b2, x3, b1);           ZK_SHIFT2(a, h, r2);
    col4(a, h, x0, a3, x1, a2, x2, b3, x3, b2);           ZK_SHIFT2(a, h, r3);
    col2(a, h, x1, a3, x3, b3);                           ZK_SHIFT2(a, h, r4);
    const uint32_t s5 = (uint32_t)a, s6 = (uint32_t)(a >> 32);
    // S' = L - H + (H K) << 32, H = r4 + s5 2^32 + s6 2^64 (s6 <= 1)
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
        "v_add_co_u32 %5, %10, %1, %19\n\t"        // e1 = d1 + q0
        "s_nop 0\n\t"
        "v_subb_co_u32 %2, %9, %13, %17, %9\n\t"   // d2 = r2 - s6 - b
        "v_addc_co_u32 %6, %10, %2, %20, %10\n\t"  // e2 = d2 + q1 + c
        "s_nop 0\n\t"
        "v_subb_co_u32 %3, %9, %14, 0, %9\n\t"     // d3
        "v_addc_co_u32 %7, %10, %3, %21, %10\n\t"  // e3 = d3 + q2 + c
        "s_nop 0\n\t"
        "v_subb_co_u32 %4, %9, 0, 0, %9\n\t"       // dm = -b
        "v_addc_co_u32 %8, %10, %4, 0, %10"        // e4 = bit 128 of S'
        : "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "=&v"(dm), "=&v"(e1), "=&v"(e2), "=&v"(e3), "=&v"(e4), "=&s"(sB),
          "=&s"(sC)
        : "v"(r0), "v"(r1), "v"(r2), "v"(r3), "v"(r4), "v"(s5), "v"(s6), "v"(0u), "v"(q0), "v"(q1), "v"(q2));
    return pre_fold(d0, e1, e2, e3, e4, 0u);
}
template <int V>
__device__ __forceinline__ fe fmul_variant(fe a, fe b, const uint32_t *W = nullptr) {
    if constexpr (V == 0) return fe_mul(a, b);
    if constexpr (V == 3 || V == 4) return fe_mul_pre(a, W);
    if constexpr (V == 5) return fe_mul_w2(a, fe{join32(W[0], W[4]), join32(W[8], W[12])}, fe{join32(W[2], W[6]), join32(W[10], W[14])});
    uint32_t r[8];
    mul_wide(a, b, r);
    if constexpr (V == 1) return reduce_v1(r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
    if constexpr (V == 2) return reduce_v2(r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
}
