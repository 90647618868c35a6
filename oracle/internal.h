/* internal.h -- shared helpers of the CPU oracle (TEST INFRASTRUCTURE ONLY, see oracle.h). */
#ifndef ZKVM_ORACLE_INTERNAL_H
#define ZKVM_ORACLE_INTERNAL_H

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef unsigned __int128 u128;

/* winterfell f128: p = 2^128 - 45 * 2^40 + 1 (constants in
 * crypto/src/rescue.rs:197-233 are written as p - c). */
#define F_P ((u128)0 - (((u128)45) << 40) + 1)
#define F_C ((((u128)45) << 40) - 1) /* 2^128 mod p */
/* 3^((p-1)/2^40): the two-adic root of unity of order 2^40 (winter-math f128 GENERATOR = 3). */
#define F_TWO_ADICITY 40
#define F_GENERATOR ((u128)3)

static inline u128 f_add(u128 a, u128 b) {
    u128 s = a + b;
    if (s < a || s >= F_P) s -= F_P;
    return s;
}
static inline u128 f_sub(u128 a, u128 b) { return a >= b ? a - b : a - b + F_P; }
static inline u128 f_neg(u128 a) { return a ? F_P - a : 0; }

static inline void mul_wide(u128 a, u128 b, u128 *hi, u128 *lo) {
    const u128 M = (u128)UINT64_MAX;
    uint64_t a0 = (uint64_t)a, a1 = (uint64_t)(a >> 64), b0 = (uint64_t)b, b1 = (uint64_t)(b >> 64);
    u128 p00 = (u128)a0 * b0, p01 = (u128)a0 * b1, p10 = (u128)a1 * b0, p11 = (u128)a1 * b1;
    u128 mid = (p00 >> 64) + (p01 & M) + (p10 & M);
    *lo = (p00 & M) | (mid << 64);
    *hi = p11 + (p01 >> 64) + (p10 >> 64) + (mid >> 64);
}

/* a * b mod p: fold the high half with 2^128 = C (mod p), C < 2^46.  lo + hi*C = s + top*2^128 with
 * top < 2^47; one more fold of top, whose carry (at most one) is again worth C. */
static inline u128 f_mul(u128 a, u128 b) {
    u128 hi, lo;
    mul_wide(a, b, &hi, &lo);
    const uint64_t C64 = (uint64_t)F_C;
    const u128 t0 = (u128)(uint64_t)hi * C64, t1 = (u128)(uint64_t)(hi >> 64) * C64;
    const u128 s1 = lo + t0;
    const u128 s2 = s1 + (t1 << 64);
    const uint64_t top = (uint64_t)(t1 >> 64) + (uint64_t)(s1 < lo) + (uint64_t)(s2 < s1);
    u128 r = s2 + (u128)top * C64;
    if (r < s2) r += F_C;
    if (r >= F_P) r -= F_P;
    return r;
}

static inline u128 f_exp(u128 b, u128 e) {
    u128 r = 1;
    while (e) {
        if (e & 1) r = f_mul(r, b);
        b = f_mul(b, b);
        e >>= 1;
    }
    return r;
}
static inline u128 f_inv(u128 a) { return f_exp(a, F_P - 2); } /* inv(0) = 0 like winterfell */
/* in-place Montgomery batch inversion (winter-math batch_inversion): one f_inv for n values (all nonzero) */
static inline void f_batch_inv(u128 *v, size_t n) {
    if (!n) return;
    u128 *pre = (u128 *)malloc(n * sizeof(u128));
    u128 acc = 1;
    for (size_t i = 0; i < n; i++) {
        pre[i] = acc;
        acc = f_mul(acc, v[i]);
    }
    u128 inv = f_inv(acc);
    for (size_t i = n; i-- > 0;) {
        const u128 vi = v[i];
        v[i] = f_mul(inv, pre[i]);
        inv = f_mul(inv, vi);
    }
    free(pre);
}

static inline u128 f_root_of_unity(unsigned log_n) {
    u128 r = f_exp(F_GENERATOR, (F_P - 1) >> F_TWO_ADICITY);
    for (unsigned i = log_n; i < F_TWO_ADICITY; i++) r = f_mul(r, r);
    return r;
}

static inline u128 ld(const void *p) {
    u128 v;
    memcpy(&v, p, 16);
    return v;
}
static inline void st(void *p, u128 v) { memcpy(p, &v, 16); }

static inline unsigned ilog2_sz(size_t n) {
    unsigned r = 0;
    while (((size_t)1 << r) < n) r++;
    return r;
}

/* NTT helpers (field_blake.c) */
void ntt_natural(u128 *a, size_t n, u128 w);
void eval_coset_u(const u128 *coeffs, size_t m, size_t size, u128 offset, u128 *out);
void interp_coset_u(u128 *vals, size_t size, u128 offset);
u128 poly_eval(const u128 *c, size_t m, u128 x);

/* BLAKE3 helpers */
void blake3_hash_elems(const u128 *e, size_t k, uint8_t out[32]);
void blake3_merge_with_int(const uint8_t seed[32], uint64_t v, uint8_t out[32]);
/* full node array: nodes[1] = root; nodes has 2*num_leaves digests, leaves separate */
uint8_t *merkle_build(const uint8_t *leaves, size_t num_leaves);

/* AIR helpers (air.c) */
void air_eval_u(const u128 *cur, const u128 *nxt, const u128 *per, uint32_t lwe, u128 delta, u128 *out);
void air_periodic_u(unsigned step16, u128 *out9);


/* winter-air AirContext::num_constraint_composition_columns for ProcessorAir (prover.c) */
size_t or_num_comp_cols(size_t n);

#endif
