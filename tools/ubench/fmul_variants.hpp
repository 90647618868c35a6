// candidate device multiplies for tools/ubench/fmul_lab.hip (variant 0 = the library's fe_mul)
#pragma once
#define FMUL_NVARIANTS 3
static const char *fmul_variant_name(int v) {
    static const char *n[] = {"library fe_mul", "v1: U = T + C final step", "v2: independent fold products, mask final step"};
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

template <int V>
__device__ __forceinline__ fe fmul_variant(fe a, fe b) {
    if constexpr (V == 0) return fe_mul(a, b);
    uint32_t r[8];
    mul_wide(a, b, r);
    if constexpr (V == 1) return reduce_v1(r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
    if constexpr (V == 2) return reduce_v2(r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
}
