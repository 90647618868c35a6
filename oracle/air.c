/*
 * air.c -- oracle: ProcessorAir::evaluate_transition and its periodic columns.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 *   evaluate_transition ........ air/src/lib.rs:104-168
 *   enforce_* .................. air/src/constrains.rs:95-216
 *   selector flags ............. air/src/flags.rs:37-91  (b0 = col 5 = opcode MSB ... b4 = col 1)
 *   ServerKey arithmetic ....... fhe/src/server_key.rs:78-124
 *   periodic columns ........... air/src/lib.rs:201-225 (CYCLE_MASK) + rescue.rs:120-136 (ARK)
 * Written as a literal restatement of the reference's formulas (no algebraic shortcuts), so that
 * it can serve as the checker for the optimised GPU kernel.
 */
#include "ext.h"
#include "internal.h"
#include "rescue_consts.h"

static u128 mds(const uint64_t m[16][2], unsigned i) { return ((u128)m[i][1] << 64) | m[i][0]; }
static u128 not_(u128 b) { return f_sub(1, b); }

void air_periodic_u(unsigned step16, u128 *out9) {
    unsigned r = step16 % 16;
    out9[0] = r < 14 ? 1 : 0; /* CYCLE_MASK */
    for (int c = 0; c < 8; c++) out9[1 + c] = ((u128)OR_ARK[8 * r + c][1] << 64) | OR_ARK[8 * r + c][0];
}

void or_air_periodic_row(uint32_t step16, void *out9) {
    u128 v[9];
    air_periodic_u(step16, v);
    memcpy(out9, v, sizeof v);
}

void air_eval_u(const u128 *cur, const u128 *nxt, const u128 *per, uint32_t lwe, u128 delta, u128 *out) {
#define S(i) cur[12 + (i)]
#define SN(i) nxt[12 + (i)]
    const u128 b0 = cur[5], b1 = cur[4], b2 = cur[3], b3 = cur[2], b4 = cur[1];
    u128 is_shr = b0, is_shl = b1;
    u128 is_add = f_mul(f_mul(f_mul(f_mul(not_(b0), b1), not_(b2)), not_(b3)), not_(b4));
    u128 is_sadd = f_mul(f_mul(f_mul(f_mul(not_(b0), b1), not_(b2)), b3), not_(b4));
    u128 is_add2 = f_mul(f_mul(f_mul(f_mul(not_(b0), b1), not_(b2)), b3), b4);
    u128 is_mul = f_mul(f_mul(f_mul(f_mul(not_(b0), b1), not_(b2)), not_(b3)), b4);
    u128 is_smul = f_mul(f_mul(f_mul(f_mul(not_(b0), b1), b2), not_(b3)), not_(b4));
    u128 is_push = f_mul(f_mul(f_mul(f_mul(b0, not_(b1)), not_(b2)), not_(b3)), not_(b4));
    u128 is_read = f_mul(f_mul(f_mul(f_mul(b0, not_(b1)), not_(b2)), not_(b3)), b4);
    u128 is_read2 = f_mul(f_mul(f_mul(f_mul(b0, not_(b1)), not_(b2)), b3), not_(b4));
    u128 is_noop = f_mul(f_mul(f_mul(f_mul(not_(b0), not_(b1)), not_(b2)), not_(b3)), not_(b4));
    u128 opcode = f_add(f_add(f_add(f_add(f_mul(b0, 16), f_mul(b1, 8)), f_mul(b2, 4)), f_mul(b3, 2)), b4);

    /* 0: clk' - (clk + 1) */
    out[0] = f_sub(nxt[0], f_add(cur[0], 1));
    /* 1: (d' - d - shr + shl) - read2*4 + add2*4 */
    out[1] = f_add(f_sub(f_add(f_sub(f_sub(nxt[11], cur[11]), is_shr), is_shl), f_mul(is_read2, 4)), f_mul(is_add2, 4));
    /* 2: shr * shl */
    out[2] = f_mul(is_shr, is_shl);
    /* 3: add */
    out[3] = f_mul(is_add, f_sub(SN(0), f_add(S(0), S(1))));
    /* 4: sadd -- server_key.scalar_add(s0, ct = s[1..1+L]) vs s'[0..L] */
    {
        u128 acc = 0;
        for (uint32_t i = 0; i < lwe; i++) {
            u128 triv = i == lwe - 1 ? f_mul(delta, S(0)) : 0; /* encrypt_trivial: [0]*k ++ [delta*m] */
            acc = f_add(acc, f_sub(SN(i), f_add(S(1 + i), triv)));
        }
        out[4] = f_mul(is_sadd, acc);
    }
    /* 5: add2 -- server_key.add(s[0..L], s[L..]) (zip takes L) vs s'[0..L] */
    {
        u128 acc = 0;
        for (uint32_t i = 0; i < lwe; i++) acc = f_add(acc, f_sub(SN(i), f_add(S(i), S(lwe + i))));
        out[5] = f_mul(is_add2, acc);
    }
    /* 6: mul */
    out[6] = f_mul(is_mul, f_sub(SN(0), f_mul(S(0), S(1))));
    /* 7: smul */
    {
        u128 acc = 0;
        for (uint32_t i = 0; i < lwe; i++) acc = f_add(acc, f_sub(SN(i), f_mul(S(1 + i), S(0))));
        out[7] = f_mul(is_smul, acc);
    }
    /* 8..11: push / read / read2 / noop */
    out[8] = f_mul(is_push, f_sub(SN(1), S(0)));
    out[9] = f_mul(is_read, f_sub(SN(1), S(0)));
    out[10] = f_mul(is_read2, f_sub(SN(5), S(0)));
    out[11] = f_mul(is_noop, f_sub(SN(0), S(0)));
    /* 12..15: hash round (constrains.rs:182-209) */
    {
        const u128 hash_flag = per[0], *ark = per + 1, h0 = cur[6];
        u128 s0[4], s1[4], t[4];
        for (int i = 0; i < 4; i++) s0[i] = f_exp(cur[7 + i], 3);
        for (int i = 0; i < 4; i++) {
            t[i] = 0;
            for (int j = 0; j < 4; j++) t[i] = f_add(t[i], f_mul(mds(OR_MDS, 4 * i + j), s0[j]));
        }
        for (int i = 0; i < 4; i++) s0[i] = f_add(t[i], ark[i]);
        s0[0] = f_add(s0[0], opcode);
        s0[1] = f_add(s0[1], f_mul(SN(0), is_push));
        for (int i = 0; i < 4; i++) s1[i] = f_sub(nxt[7 + i], ark[4 + i]);
        for (int i = 0; i < 4; i++) {
            t[i] = 0;
            for (int j = 0; j < 4; j++) t[i] = f_add(t[i], f_mul(mds(OR_INV_MDS, 4 * i + j), s1[j]));
        }
        for (int i = 0; i < 4; i++) s1[i] = f_exp(t[i], 3);
        for (int i = 0; i < 4; i++) out[12 + i] = f_mul(f_mul(f_sub(s1[i], s0[i]), hash_flag), h0);
        /* 16..19: hash copy (constrains.rs:211-216) */
        u128 nf = not_(hash_flag);
        out[16] = f_mul(f_mul(f_sub(nxt[7], cur[7]), nf), h0);
        out[17] = f_mul(f_mul(f_sub(nxt[8], cur[8]), nf), h0);
        out[18] = f_mul(f_mul(nxt[9], nf), h0);
        out[19] = f_mul(f_mul(nxt[10], nf), h0);
    }
#undef S
#undef SN
}

void or_air_eval_transition(const void *cur, const void *nxt, const void *periodic9, uint32_t lwe_size,
                            uint32_t delta, void *out20) {
    u128 c[28], n[28], p[9], o[20];
    memcpy(c, cur, sizeof c);
    memcpy(n, nxt, sizeof n);
    memcpy(p, periodic9, sizeof p);
    air_eval_u(c, n, p, lwe_size, (u128)delta, o);
    memcpy(out20, o, sizeof o);
}

/* The same transition evaluated over E (evaluate_transition<E> with E = QuadExtension<f128>, as the
 * verifier calls it at the out-of-domain point, air/src/lib.rs:104-168).  Same formula order as
 * air_eval_u, every operand lifted to e2. */
static e2 nE(e2 b) { return e2_sub(e2_base(1), b); }
static e2 mE(e2 x, e2 y) { return e2_mul(x, y); }
void air_eval_e(const e2 *cur, const e2 *nxt, const e2 *per, uint32_t lwe, u128 delta, e2 *out) {
#define S(i) cur[12 + (i)]
#define SN(i) nxt[12 + (i)]
#define C_(v) e2_base((u128)(v))
    const e2 b0 = cur[5], b1 = cur[4], b2 = cur[3], b3 = cur[2], b4 = cur[1];
    e2 is_shr = b0, is_shl = b1;
    e2 is_add = mE(mE(mE(mE(nE(b0), b1), nE(b2)), nE(b3)), nE(b4));
    e2 is_sadd = mE(mE(mE(mE(nE(b0), b1), nE(b2)), b3), nE(b4));
    e2 is_add2 = mE(mE(mE(mE(nE(b0), b1), nE(b2)), b3), b4);
    e2 is_mul = mE(mE(mE(mE(nE(b0), b1), nE(b2)), nE(b3)), b4);
    e2 is_smul = mE(mE(mE(mE(nE(b0), b1), b2), nE(b3)), nE(b4));
    e2 is_push = mE(mE(mE(mE(b0, nE(b1)), nE(b2)), nE(b3)), nE(b4));
    e2 is_read = mE(mE(mE(mE(b0, nE(b1)), nE(b2)), nE(b3)), b4);
    e2 is_read2 = mE(mE(mE(mE(b0, nE(b1)), nE(b2)), b3), nE(b4));
    e2 is_noop = mE(mE(mE(mE(nE(b0), nE(b1)), nE(b2)), nE(b3)), nE(b4));
    e2 opcode = e2_add(e2_add(e2_add(e2_add(e2_mulb(b0, 16), e2_mulb(b1, 8)), e2_mulb(b2, 4)), e2_mulb(b3, 2)), b4);

    out[0] = e2_sub(nxt[0], e2_add(cur[0], C_(1)));
    out[1] = e2_add(e2_sub(e2_add(e2_sub(e2_sub(nxt[11], cur[11]), is_shr), is_shl), e2_mulb(is_read2, 4)),
                    e2_mulb(is_add2, 4));
    out[2] = mE(is_shr, is_shl);
    out[3] = mE(is_add, e2_sub(SN(0), e2_add(S(0), S(1))));
    {
        e2 acc = C_(0);
        for (uint32_t i = 0; i < lwe; i++) {
            e2 triv = i == lwe - 1 ? e2_mulb(S(0), delta) : C_(0);
            acc = e2_add(acc, e2_sub(SN(i), e2_add(S(1 + i), triv)));
        }
        out[4] = mE(is_sadd, acc);
    }
    {
        e2 acc = C_(0);
        for (uint32_t i = 0; i < lwe; i++) acc = e2_add(acc, e2_sub(SN(i), e2_add(S(i), S(lwe + i))));
        out[5] = mE(is_add2, acc);
    }
    out[6] = mE(is_mul, e2_sub(SN(0), mE(S(0), S(1))));
    {
        e2 acc = C_(0);
        for (uint32_t i = 0; i < lwe; i++) acc = e2_add(acc, e2_sub(SN(i), mE(S(1 + i), S(0))));
        out[7] = mE(is_smul, acc);
    }
    out[8] = mE(is_push, e2_sub(SN(1), S(0)));
    out[9] = mE(is_read, e2_sub(SN(1), S(0)));
    out[10] = mE(is_read2, e2_sub(SN(5), S(0)));
    out[11] = mE(is_noop, e2_sub(SN(0), S(0)));
    {
        const e2 hash_flag = per[0], *ark = per + 1, h0 = cur[6];
        e2 s0[4], s1[4], t[4];
        for (int i = 0; i < 4; i++) s0[i] = e2_exp(cur[7 + i], 3);
        for (int i = 0; i < 4; i++) {
            t[i] = C_(0);
            for (int j = 0; j < 4; j++) t[i] = e2_add(t[i], e2_mulb(s0[j], mds(OR_MDS, 4 * i + j)));
        }
        for (int i = 0; i < 4; i++) s0[i] = e2_add(t[i], ark[i]);
        s0[0] = e2_add(s0[0], opcode);
        s0[1] = e2_add(s0[1], mE(SN(0), is_push));
        for (int i = 0; i < 4; i++) s1[i] = e2_sub(nxt[7 + i], ark[4 + i]);
        for (int i = 0; i < 4; i++) {
            t[i] = C_(0);
            for (int j = 0; j < 4; j++) t[i] = e2_add(t[i], e2_mulb(s1[j], mds(OR_INV_MDS, 4 * i + j)));
        }
        for (int i = 0; i < 4; i++) s1[i] = e2_exp(t[i], 3);
        for (int i = 0; i < 4; i++) out[12 + i] = mE(mE(e2_sub(s1[i], s0[i]), hash_flag), h0);
        e2 nf = nE(hash_flag);
        out[16] = mE(mE(e2_sub(nxt[7], cur[7]), nf), h0);
        out[17] = mE(mE(e2_sub(nxt[8], cur[8]), nf), h0);
        out[18] = mE(mE(nxt[9], nf), h0);
        out[19] = mE(mE(nxt[10], nf), h0);
    }
#undef C_
#undef S
#undef SN
}

void or_e2_mul(const void *x, const void *y, void *out) {
    const uint8_t *a = (const uint8_t *)x, *b = (const uint8_t *)y;
    e2 r = e2_mul(e2_make(ld(a), ld(a + 16)), e2_make(ld(b), ld(b + 16)));
    st(out, r.a);
    st((uint8_t *)out + 16, r.b);
}
void or_e2_inv(const void *x, void *out) {
    const uint8_t *a = (const uint8_t *)x;
    e2 r = e2_inv(e2_make(ld(a), ld(a + 16)));
    st(out, r.a);
    st((uint8_t *)out + 16, r.b);
}
