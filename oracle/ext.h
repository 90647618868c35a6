/*
 * ext.h -- oracle: the quadratic extension E = F[X]/(X^2 - X - 1) of the f128 field (winter-math
 * `ExtensibleField<2> for f128::BaseElement`; FieldExtension::Quadratic in ProofOptions,
 * vm/src/lib.rs:20 uses None).  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Every E-valued quantity of the prover/verifier is an e2 = a + b*X.  Base-field values carry b = 0
 * and the operations short-circuit on them, so FieldExtension::None (k = 1) runs the same code with
 * base-field cost; only coin draws, hashing and serialization look at k.
 *   mul: (a0 + a1 X)(b0 + b1 X) = (a0 b0 + a1 b1) + ((a0 + a1)(b0 + b1) - a0 b0) X      (X^2 = X + 1)
 *   inv: (a0 + a1 X)^-1 = ((a0 + a1) - a1 X) / (a0^2 + a0 a1 - a1^2)
 */
#ifndef ORACLE_EXT_H
#define ORACLE_EXT_H
#include "internal.h"

typedef struct {
    u128 a, b;
} e2;

static inline e2 e2_base(u128 v) {
    e2 r = {v, 0};
    return r;
}
static inline e2 e2_make(u128 a, u128 b) {
    e2 r = {a, b};
    return r;
}
static inline e2 e2_add(e2 x, e2 y) { return e2_make(f_add(x.a, y.a), f_add(x.b, y.b)); }
static inline e2 e2_sub(e2 x, e2 y) { return e2_make(f_sub(x.a, y.a), f_sub(x.b, y.b)); }
static inline e2 e2_mul(e2 x, e2 y) {
    if (!x.b && !y.b) return e2_base(f_mul(x.a, y.a));
    const u128 z = f_mul(x.a, y.a);
    return e2_make(f_add(z, f_mul(x.b, y.b)), f_sub(f_mul(f_add(x.a, x.b), f_add(y.a, y.b)), z));
}
static inline e2 e2_mulb(e2 x, u128 s) { return e2_make(f_mul(x.a, s), x.b ? f_mul(x.b, s) : 0); }
static inline e2 e2_inv(e2 x) {
    if (!x.b) return e2_base(f_inv(x.a));
    const u128 d = f_sub(f_add(f_mul(x.a, x.a), f_mul(x.a, x.b)), f_mul(x.b, x.b));
    const u128 di = f_inv(d);
    return e2_make(f_mul(f_add(x.a, x.b), di), f_neg(f_mul(x.b, di)));
}
static inline e2 e2_mulX(e2 v) { return e2_make(v.b, f_add(v.a, v.b)); } /* X * (a + bX) = b + (a + b) X */
static inline int e2_eq(e2 x, e2 y) { return x.a == y.a && x.b == y.b; }
static inline e2 e2_exp(e2 x, uint64_t e) {
    e2 r = e2_base(1);
    while (e) {
        if (e & 1) r = e2_mul(r, x);
        x = e2_mul(x, x);
        e >>= 1;
    }
    return r;
}
/* sum_t c[t] x^t for base coefficients at an E point (Horner) */
static inline e2 poly_eval_e(const u128 *c, size_t m, e2 x) {
    e2 acc = e2_base(0);
    for (size_t t = m; t-- > 0;) acc = e2_add(e2_mul(acc, x), e2_base(c[t]));
    return acc;
}
/* the first k components of n E values, as base elements (hash / serialization order) */
static inline void e2_flatten(const e2 *v, size_t n, int k, u128 *out) {
    for (size_t i = 0; i < n; i++) {
        out[k * i] = v[i].a;
        if (k == 2) out[k * i + 1] = v[i].b;
    }
}
static inline void e2_hash(const e2 *v, size_t n, int k, uint8_t out[32]) {
    u128 *flat = (u128 *)malloc((n ? n : 1) * k * 16);
    e2_flatten(v, n, k, flat);
    blake3_hash_elems(flat, n * k, out);
    free(flat);
}
/* ProcessorAir::evaluate_transition over E (air.c) */
void air_eval_e(const e2 *cur, const e2 *nxt, const e2 *per, uint32_t lwe, u128 delta, e2 *out);
#endif
