/*
 * prover.c -- oracle: the STARK prove path of prover/src/lib.rs:40-77 (ExecutionProver, an
 * `impl winterfell::Prover`) as executed by winterfell 0.9.0 `Prover::prove` / generate_proof.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  PARITY UNPINNED at the winterfell boundary: the
 * protocol choices below follow the published winterfell 0.9 design and are listed one by one in
 * DESIGN.md "Protocol profile" (P1..P14); each is marked [Pk] where it is made.
 *
 * Deliberately simple: row-major LDE, full-size zero-padded NTTs, one inversion per point where
 * that is clearer than a batched form.  Speed is irrelevant; obviousness is the point.
 */
#include <stdio.h>

#include "ext.h"
#include "internal.h"

#define W 28 /* ProcessorAir trace width (vm/src/processor/mod.rs:76-84) */
#define NUM_TCONS 20
#define NUM_ASSERTS 22
#define CE_BLOWUP 8 /* max TransitionConstraintDegree::min_blowup_factor (air/src/lib.rs:69-90) */

/* ----------------------------------------------------------------- public coin [P2] */
typedef struct {
    uint8_t seed[32];
    uint64_t counter;
} coin_t;

static void coin_init(coin_t *c, const u128 *elems, size_t k) {
    blake3_hash_elems(elems, k, c->seed);
    c->counter = 0;
}
static void coin_reseed(coin_t *c, const uint8_t d[32]) {
    uint8_t out[32];
    or_blake3_merge(c->seed, d, out);
    memcpy(c->seed, out, 32);
    c->counter = 0;
}
static void coin_next(coin_t *c, uint8_t out[32]) {
    c->counter++;
    blake3_merge_with_int(c->seed, c->counter, out);
}
/* coefficients of the degree < f polynomial through (x0 * zeta^k, v[k]), zeta = w_f (interp_coset_u over
 * x0 * <w_f> with the inverses precomputed): c_m = (1/f) x0^-m sum_k v_k zeta^-km */
static void interp_small(u128 *v, size_t f, u128 inv_x0, const u128 *zinv, u128 inv_f) {
    u128 c[16];
    for (size_t m = 0; m < f; m++) {
        u128 acc = 0;
        for (size_t k = 0; k < f; k++) acc = f_add(acc, f_mul(v[k], zinv[(k * m) & (f - 1)]));
        c[m] = acc;
    }
    u128 sc = inv_f;
    for (size_t m = 0; m < f; m++) {
        v[m] = f_mul(c[m], sc);
        sc = f_mul(sc, inv_x0);
    }
}

/* DefaultRandomCoin::draw::<E>: the first E::ELEMENT_BYTES of the next digest, retried until every
 * base component is canonical (k = 1: 16 bytes; k = 2: both 16-byte halves) */
static e2 coin_draw_e(coin_t *c, int k) {
    for (int i = 0; i < 1000; i++) {
        uint8_t d[32];
        coin_next(c, d);
        const u128 a = ld(d);
        if (k == 1) {
            if (a < F_P) return e2_base(a);
        } else {
            const u128 b = ld(d + 16);
            if (a < F_P && b < F_P) return e2_make(a, b);
        }
    }
    return e2_base(0);
}

/* ----------------------------------------------------------------- byte writer */
typedef struct {
    uint8_t *p;
    size_t len, cap;
} buf_t;
static void bw(buf_t *b, const void *d, size_t n) {
    if (b->len + n > b->cap) {
        b->cap = (b->len + n) * 2 + 256;
        b->p = (uint8_t *)realloc(b->p, b->cap);
    }
    memcpy(b->p + b->len, d, n);
    b->len += n;
}
static void bw_u8(buf_t *b, uint8_t v) { bw(b, &v, 1); }
static void bw_u16(buf_t *b, uint16_t v) { bw(b, &v, 2); }
static void bw_u32(buf_t *b, uint32_t v) { bw(b, &v, 4); }
static void bw_u64(buf_t *b, uint64_t v) { bw(b, &v, 8); }

/* ----------------------------------------------------------------- batch Merkle proof [P12] */
/* winter-crypto MerkleTree::prove_batch + BatchMerkleProof::serialize_nodes. */
static void prove_batch(const uint8_t *leaves, const uint8_t *nodes, size_t nl, const uint64_t *idx, size_t k,
                        buf_t *out) {
    unsigned depth = ilog2_sz(nl);
    /* normalized indexes: sorted, unique, even */
    uint64_t *norm = (uint64_t *)malloc(k * 8);
    size_t nn = 0;
    for (size_t i = 0; i < k; i++) {
        uint64_t v = idx[i] & ~1ULL;
        size_t j = nn;
        int dup = 0;
        for (size_t t = 0; t < nn; t++)
            if (norm[t] == v) dup = 1;
        if (dup) continue;
        while (j > 0 && norm[j - 1] > v) {
            norm[j] = norm[j - 1];
            j--;
        }
        norm[j] = v;
        nn++;
    }
    uint8_t **paths = (uint8_t **)calloc(nn, sizeof(uint8_t *));
    size_t *plen = (size_t *)calloc(nn, sizeof(size_t));
    for (size_t i = 0; i < nn; i++) paths[i] = (uint8_t *)malloc(32 * (depth + 2));
    uint64_t *next = (uint64_t *)malloc(nn * 8), *cur = (uint64_t *)malloc(nn * 8);
    for (size_t i = 0; i < nn; i++) {
        for (uint64_t l = norm[i]; l < norm[i] + 2; l++) {
            int queried = 0;
            for (size_t t = 0; t < k; t++)
                if (idx[t] == l) queried = 1;
            if (!queried) memcpy(paths[i] + 32 * plen[i]++, leaves + 32 * l, 32);
        }
        next[i] = (norm[i] + nl) >> 1;
    }
    size_t nnext = nn;
    for (unsigned lvl = 1; lvl < depth; lvl++) {
        memcpy(cur, next, nnext * 8);
        size_t ncur = nnext;
        nnext = 0;
        for (size_t i = 0; i < ncur; i++) {
            uint64_t sib = cur[i] ^ 1;
            if (i + 1 < ncur && cur[i + 1] == sib)
                i++;
            else
                memcpy(paths[i] + 32 * plen[i]++, nodes + 32 * sib, 32);
            next[nnext++] = sib >> 1;
        }
    }
    bw_u8(out, (uint8_t)nn);
    for (size_t i = 0; i < nn; i++) {
        bw_u8(out, (uint8_t)plen[i]);
        bw(out, paths[i], 32 * plen[i]);
        free(paths[i]);
    }
    free(paths);
    free(plen);
    free(norm);
    free(next);
    free(cur);
}

/* Queries::new + write_into: u32 len + value bytes, u32 len + path bytes */
static void write_queries(buf_t *out, const uint8_t *vals, size_t vlen, const buf_t *paths) {
    bw_u32(out, (uint32_t)vlen);
    bw(out, vals, vlen);
    bw_u32(out, (uint32_t)paths->len);
    bw(out, paths->p, paths->len);
}

/* ----------------------------------------------------------------- AIR metadata */
/* TransitionConstraintDegree (base, has 16-cycle) of air/src/lib.rs:69-90 */
static const int DEG_BASE[NUM_TCONS] = {1, 5, 2, 6, 6, 6, 7, 7, 6, 6, 6, 6, 4, 7, 4, 4, 2, 2, 2, 2};
static const int DEG_CYC[NUM_TCONS] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1};

/* winter-air AirContext::num_constraint_composition_columns [P5] */
size_t or_num_comp_cols(size_t n) {
    size_t hi = 0;
    for (int k = 0; k < NUM_TCONS; k++) {
        size_t d = (size_t)DEG_BASE[k] * (n - 1) + (DEG_CYC[k] ? (n / 16) * 15 : 0);
        if (d > hi) hi = d;
    }
    size_t div = n - 2; /* 2 transition exemptions (air/src/lib.rs:94) */
    size_t c = (hi - div + n - 1) / n;
    return c ? c : 1;
}

/* Assertions (air/src/lib.rs:170-195) sorted by (stride, first_step, column) [P3] */
typedef struct {
    int col;
    size_t step;
    u128 value;
} assertion_t;

static size_t sorted_assertions(size_t n, const or_pub_inputs *pub, assertion_t *a) {
    size_t last = n - 2, k = 0;
    const int first_cols[12] = {0, 7, 8, 11, 12, 13, 14, 15, 16, 17, 18, 19};
    for (int i = 0; i < 12; i++) a[k++] = (assertion_t){first_cols[i], 0, 0};
    for (int i = 0; i < 2; i++) a[k++] = (assertion_t){7 + i, last, ld(pub->program_hash[i])};
    for (int i = 0; i < 8; i++) a[k++] = (assertion_t){12 + i, last, ld(pub->stack_outputs[i])};
    return k;
}

/* ----------------------------------------------------------------- prove */
int or_prove(const void *trace_v, size_t n, const or_options *opt, const or_pub_inputs *pub, uint8_t *proof_out,
             size_t *proof_len, or_record *rec, const or_dump *dump) {
    if (n < 16 || (n & (n - 1)) || !opt || !pub || !proof_len) return OR_ERR_INVALID_ARG;
    if ((opt->field_extension != 1 && opt->field_extension != 2) || opt->blowup < CE_BLOWUP || (opt->blowup & (opt->blowup - 1)) ||
        (opt->fri_folding != 2 && opt->fri_folding != 4 && opt->fri_folding != 8 && opt->fri_folding != 16) ||
        ((opt->fri_rem_max_deg + 1) & opt->fri_rem_max_deg) || opt->num_queries == 0 ||
        opt->num_queries > OR_MAX_QUERIES || pub->lwe_size == 0 || pub->lwe_size > 5)
        return OR_ERR_INVALID_ARG;
    const u128 *trace = (const u128 *)trace_v;
    const size_t B = opt->blowup, N = B * n, CE = CE_BLOWUP * n, fold = opt->fri_folding;
    if (opt->num_queries >= N) return OR_ERR_INVALID_ARG;
    const size_t C = or_num_comp_cols(n);
    const int K = (int)opt->field_extension; /* 1: FieldExtension::None, 2: Quadratic */
    const u128 offset = F_GENERATOR; /* StarkDomain offset = GENERATOR [P1] */
    const u128 g_n = f_root_of_unity(ilog2_sz(n));
    or_record R;
    memset(&R, 0, sizeof R);
    R.trace_len = (uint32_t)n;
    R.lde_len = (uint32_t)N;
    R.width = W;
    R.num_ccols = (uint32_t)C;

    /* S0: coin seed = Context::to_elements() || PublicInputs::to_elements() [P1] */
    coin_t coin;
    {
        u128 e[8 + 18];
        size_t k = 0;
        e[k++] = (u128)W << 16;                                /* TraceInfo: width | aux width | aux rands */
        e[k++] = (u128)n;                                      /* trace length */
        e[k++] = (u128)(uint64_t)F_P;                          /* modulus bytes [0..8) */
        e[k++] = (u128)(uint64_t)(F_P >> 64);                  /* modulus bytes [8..16) */
        e[k++] = ((u128)opt->field_extension << 16) | ((u128)fold << 8) | opt->fri_rem_max_deg;
        e[k++] = opt->grinding;
        e[k++] = B;
        e[k++] = opt->num_queries;
        for (int i = 0; i < 2; i++) e[k++] = ld(pub->program_hash[i]);
        for (int i = 0; i < 16; i++) e[k++] = ld(pub->stack_outputs[i]);
        coin_init(&coin, e, k);
    }

    /* S2: trace LDE + commitment (DefaultTraceLde::new) */
    u128 *polys = (u128 *)malloc(W * n * 16);
    u128 *lde = (u128 *)malloc(N * W * 16);
    uint8_t *leaves = (uint8_t *)malloc(N * 32);
    {
        u128 *col = (u128 *)malloc(N * 16);
        for (int c = 0; c < W; c++) {
            memcpy(polys + c * n, trace + c * n, n * 16);
            interp_coset_u(polys + c * n, n, 1);
            eval_coset_u(polys + c * n, n, N, offset, col);
            for (size_t i = 0; i < N; i++) lde[i * W + c] = col[i];
        }
        free(col);
        for (size_t i = 0; i < N; i++) blake3_hash_elems(lde + i * W, W, leaves + 32 * i);
    }
    uint8_t *tnodes = merkle_build(leaves, N);
    memcpy(R.trace_root, tnodes + 32, 32);
    coin_reseed(&coin, R.trace_root);

    /* S3: composition coefficients (transition then boundary) [P4], drawn in E, and evaluation */
    e2 ct[NUM_TCONS], cb[NUM_ASSERTS];
    for (int k = 0; k < NUM_TCONS; k++) st(R.coeff_t[k], (ct[k] = coin_draw_e(&coin, K)).a);
    for (int k = 0; k < NUM_ASSERTS; k++) st(R.coeff_b[k], (cb[k] = coin_draw_e(&coin, K)).a);
    assertion_t as[NUM_ASSERTS];
    sorted_assertions(n, pub, as);
    e2 *comp = (e2 *)malloc(CE * sizeof(e2));
    {
        const size_t lde_shift = N / CE;
        const u128 w_ce = f_root_of_unity(ilog2_sz(CE));
        const u128 g_last2 = f_exp(g_n, n - 2), g_last1 = f_exp(g_n, n - 1);
        /* periodic values: P_j((x)^(n/16)), P_j interpolating the 16 column values over <w_16> */
        u128 pcoef[9][16];
        for (unsigned r = 0; r < 16; r++) {
            u128 row[9];
            air_periodic_u(r, row);
            for (int j = 0; j < 9; j++) pcoef[j][r] = row[j];
        }
        for (int j = 0; j < 9; j++) interp_coset_u(pcoef[j], 16, 1);
        /* x^(n/16) = offset^(n/16) * w_128^i depends on i mod 128 only (winterfell evaluates the periodic
         * polynomials once per distinct point): a 128-row table */
        u128(*pertab)[9] = (u128(*)[9])malloc(128 * sizeof(*pertab));
        {
            u128 y = f_exp(offset, n / 16);
            const u128 w128 = f_root_of_unity(7);
            for (int r = 0; r < 128; r++) {
                for (int j = 0; j < 9; j++) pertab[r][j] = poly_eval(pcoef[j], 16, y);
                y = f_mul(y, w128);
            }
        }
        /* divisor inverses: x^n = offset^n * w_8^i takes 8 values; the boundary denominators
         * (x - 1)(x - g^(n-2)) are batch-inverted over the CE domain (winter-math batch_inversion) */
        u128 inv_xn[8];
        {
            u128 y = f_exp(offset, n);
            const u128 w8 = f_root_of_unity(3);
            for (int r = 0; r < 8; r++) {
                inv_xn[r] = f_inv(f_sub(y, 1));
                y = f_mul(y, w8);
            }
        }
        u128 *bden = (u128 *)malloc(CE * sizeof(u128));
        {
            u128 x = offset;
            for (size_t i = 0; i < CE; i++) {
                bden[i] = f_mul(f_sub(x, 1), f_sub(x, g_last2));
                x = f_mul(x, w_ce);
            }
            f_batch_inv(bden, CE);
        }
        u128 x = offset;
        for (size_t i = 0; i < CE; i++) {
            const u128 *cur = lde + (i * lde_shift) * W, *nxt = lde + ((i * lde_shift + B) % N) * W;
            u128 ev[NUM_TCONS];
            air_eval_u(cur, nxt, pertab[i & 127], pub->lwe_size, pub->delta, ev);
            e2 t = e2_base(0);
            for (int k = 0; k < NUM_TCONS; k++) t = e2_add(t, e2_mulb(ct[k], ev[k]));
            /* transition divisor (x^n - 1) / ((x - g^(n-2)) (x - g^(n-1))) [P6]: multiply by its inverse */
            const u128 xa = f_sub(x, g_last2);
            e2 acc = e2_mulb(t, f_mul(f_mul(xa, f_sub(x, g_last1)), inv_xn[i & 7]));
            /* boundary groups keyed by (stride, step): (0,0) then (0,n-2) [P3] */
            e2 b0 = e2_base(0), b1 = e2_base(0);
            for (int k = 0; k < NUM_ASSERTS; k++) {
                e2 v = e2_mulb(cb[k], f_sub(cur[as[k].col], as[k].value));
                if (as[k].step == 0) b0 = e2_add(b0, v);
                else b1 = e2_add(b1, v);
            }
            acc = e2_add(acc, e2_mulb(b0, f_mul(bden[i], xa)));                 /* / (x - 1) */
            acc = e2_add(acc, e2_mulb(b1, f_mul(bden[i], f_sub(x, 1))));        /* / (x - g^(n-2)) */
            comp[i] = acc;
            x = f_mul(x, w_ce);
        }
        free(bden);
        free(pertab);
    }
    if (dump && dump->composition)
        for (size_t i = 0; i < CE; i++) st((uint8_t *)dump->composition + 16 * i, comp[i].a);

    /* S4: constraint commitment: interpolate each E component over the CE coset, segment into C
     * columns of E polynomials (base polys (col, j) at cpolys[(col*K + j)*n]) [P5]; a leaf is the row
     * of C E values, i.e. C*K base elements */
    const size_t CK = C * K;
    u128 *cpolys = (u128 *)calloc(CK * n, 16);
    u128 *clde = (u128 *)malloc(N * CK * 16);
    uint8_t *cleaves = (uint8_t *)malloc(N * 32);
    int degree_ok = 1;
    {
        u128 *coef = (u128 *)malloc(CE * 16);
        u128 *col = (u128 *)malloc(N * 16);
        for (int j = 0; j < K; j++) {
            for (size_t i = 0; i < CE; i++) coef[i] = j ? comp[i].b : comp[i].a;
            interp_coset_u(coef, CE, offset);
            for (size_t k = C * n; k < CE; k++)
                if (coef[k]) degree_ok = 0; /* composition degree must be < C*n */
            for (size_t c = 0; c < C; c++) {
                u128 *pc = cpolys + (c * K + j) * n;
                memcpy(pc, coef + c * n, n * 16);
                eval_coset_u(pc, n, N, offset, col);
                for (size_t i = 0; i < N; i++) clde[i * CK + c * K + j] = col[i];
            }
        }
        free(col);
        free(coef);
        for (size_t i = 0; i < N; i++) blake3_hash_elems(clde + i * CK, CK, cleaves + 32 * i);
    }
    uint8_t *cnodes = merkle_build(cleaves, N);
    memcpy(R.constraint_root, cnodes + 32, 32);
    coin_reseed(&coin, R.constraint_root);

    /* S5: OOD point (in E) and frame [P7] */
    const e2 z = coin_draw_e(&coin, K), zg = e2_mulb(z, g_n);
    st(R.z, z.a);
    e2 ood[2 * W], oodc[OR_MAX_CCOLS];
    for (int c = 0; c < W; c++) {
        ood[c] = poly_eval_e(polys + c * n, n, z);
        ood[W + c] = poly_eval_e(polys + c * n, n, zg);
        st(R.ood_trace_z[c], ood[c].a);
        st(R.ood_trace_zg[c], ood[W + c].a);
    }
    {
        uint8_t h[32];
        e2_hash(ood, 2 * W, K, h);
        coin_reseed(&coin, h);
    }
    for (size_t c = 0; c < C; c++) {
        oodc[c] = poly_eval_e(cpolys + c * K * n, n, z);
        if (K == 2) oodc[c] = e2_add(oodc[c], e2_mulX(poly_eval_e(cpolys + (c * K + 1) * n, n, z)));
        st(R.ood_constraints[c], oodc[c].a);
    }
    {
        uint8_t h[32];
        e2_hash(oodc, C, K, h);
        coin_reseed(&coin, h);
    }
    /* DEEP coefficients [P8] and DEEP evaluations over the LDE domain (evaluation form) */
    e2 at[W], ac[OR_MAX_CCOLS];
    for (int c = 0; c < W; c++) st(R.deep_t[c], (at[c] = coin_draw_e(&coin, K)).a);
    for (size_t c = 0; c < C; c++) st(R.deep_c[c], (ac[c] = coin_draw_e(&coin, K)).a);
    e2 *deep = (e2 *)malloc(N * sizeof(e2));
    {
        const u128 w_n = f_root_of_unity(ilog2_sz(N));
        /* 1/((x - z)(x - zg)) for all x: batch inversion of the E products via their base norms
         * (N(a + bX) = a^2 + ab - b^2; a base value is its own norm's square root case b = 0) */
        e2 *dden = (e2 *)malloc(N * sizeof(e2));
        u128 *nrm = (u128 *)malloc(N * sizeof(u128));
        {
            u128 x = offset;
            for (size_t i = 0; i < N; i++) {
                const e2 xe = e2_base(x);
                const e2 d = e2_mul(e2_sub(xe, z), e2_sub(xe, zg));
                dden[i] = d;
                nrm[i] = d.b ? f_sub(f_add(f_mul(d.a, d.a), f_mul(d.a, d.b)), f_mul(d.b, d.b)) : d.a;
                x = f_mul(x, w_n);
            }
            f_batch_inv(nrm, N);
            for (size_t i = 0; i < N; i++) {  /* d^-1 = conj(d) / N(d), conj(a + bX) = (a + b) - bX */
                const e2 d = dden[i];
                dden[i] = d.b ? e2_make(f_mul(f_add(d.a, d.b), nrm[i]), f_neg(f_mul(d.b, nrm[i]))) : e2_base(nrm[i]);
            }
            free(nrm);
        }
        u128 x = offset;
        for (size_t i = 0; i < N; i++) {
            e2 s1 = e2_base(0), s2 = e2_base(0);
            for (int c = 0; c < W; c++) {
                const e2 v = e2_base(lde[i * W + c]);
                s1 = e2_add(s1, e2_mul(at[c], e2_sub(v, ood[c])));
                s2 = e2_add(s2, e2_mul(at[c], e2_sub(v, ood[W + c])));
            }
            for (size_t c = 0; c < C; c++) {
                const e2 h = e2_make(clde[i * CK + c * K], K == 2 ? clde[i * CK + c * K + 1] : 0);
                s1 = e2_add(s1, e2_mul(ac[c], e2_sub(h, oodc[c])));
            }
            const e2 xe = e2_base(x);
            /* s1/(x - z) + s2/(x - zg) = (s1 (x - zg) + s2 (x - z)) / ((x - z)(x - zg)) */
            deep[i] = e2_mul(e2_add(e2_mul(s1, e2_sub(xe, zg)), e2_mul(s2, e2_sub(xe, z))), dden[i]);
            x = f_mul(x, w_n);
        }
        free(dden);
    }
    if (dump && dump->deep)
        for (size_t i = 0; i < N; i++) st((uint8_t *)dump->deep + 16 * i, deep[i].a);

    /* S6: FRI over E [P9, P10] */
    size_t max_rem = (size_t)(opt->fri_rem_max_deg + 1) * B, nl = 0;
    for (size_t s = N; s > max_rem; s /= fold) nl++;
    if (nl > OR_MAX_FRI_LAYERS) return OR_ERR_INVALID_ARG;
    R.num_fri_layers = (uint32_t)nl;
    e2 *layer_vals[OR_MAX_FRI_LAYERS]; /* transposed: row r = [e[r + k*L/fold]] */
    uint8_t *layer_leaves[OR_MAX_FRI_LAYERS], *layer_nodes[OR_MAX_FRI_LAYERS];
    size_t layer_rows[OR_MAX_FRI_LAYERS];
    e2 *ev = deep;
    size_t L = N;
    for (size_t l = 0; l < nl; l++) {
        size_t rows = L / fold;
        e2 *tv = (e2 *)malloc(L * sizeof(e2));
        for (size_t r = 0; r < rows; r++)
            for (size_t k = 0; k < fold; k++) tv[r * fold + k] = ev[r + k * rows];
        uint8_t *lv = (uint8_t *)malloc(rows * 32);
        for (size_t r = 0; r < rows; r++) e2_hash(tv + r * fold, fold, K, lv + 32 * r);
        uint8_t *nodes = merkle_build(lv, rows);
        memcpy(R.fri_roots[l], nodes + 32, 32);
        coin_reseed(&coin, R.fri_roots[l]);
        const e2 alpha = coin_draw_e(&coin, K);
        st(R.fri_alphas[l], alpha.a);
        /* degree-respecting projection: p_r interpolates (offset*w_L^r*zeta^k, tv[r][k]); next[r] = p_r(alpha) */
        e2 *nx = (e2 *)malloc(rows * sizeof(e2));
        /* x_r = offset * w_L^r; x_r^-1 advances by w_L^-1; the fold-point DFT uses zeta^-t, zeta = w_fold */
        const u128 wl_inv = f_inv(f_root_of_unity(ilog2_sz(L))), inv_f = f_inv((u128)fold);
        u128 zinv[16];
        zinv[0] = 1;
        for (size_t t = 1; t < fold; t++) zinv[t] = f_mul(zinv[t - 1], f_inv(f_root_of_unity(ilog2_sz(fold))));
        u128 xr_inv = f_inv(offset);
        for (size_t r = 0; r < rows; r++) {
            u128 va[16], vb[16];
            for (size_t k = 0; k < fold; k++) {
                va[k] = tv[r * fold + k].a;
                vb[k] = tv[r * fold + k].b;
            }
            interp_small(va, fold, xr_inv, zinv, inv_f); /* coefficients of p_r in x, per E component */
            if (K == 2) interp_small(vb, fold, xr_inv, zinv, inv_f);
            e2 acc = e2_base(0);
            for (size_t m = fold; m-- > 0;) acc = e2_add(e2_mul(acc, alpha), e2_make(va[m], K == 2 ? vb[m] : 0));
            nx[r] = acc;
            xr_inv = f_mul(xr_inv, wl_inv);
        }
        layer_vals[l] = tv;
        layer_leaves[l] = lv;
        layer_nodes[l] = nodes;
        layer_rows[l] = rows;
        if (l == 0 && dump && dump->fri_layer1)
            for (size_t r = 0; r < rows; r++) st((uint8_t *)dump->fri_layer1 + 16 * r, nx[r].a);
        if (ev != deep) free(ev);
        ev = nx;
        L = rows;
    }
    /* remainder: interpolate over offset*<w_L>, keep L/blowup coefficients (in E), commit by hash */
    e2 rem[OR_MAX_REMAINDER];
    size_t rl = L / B;
    {
        if (rl > OR_MAX_REMAINDER) return OR_ERR_INVALID_ARG;
        u128 *ra = (u128 *)malloc(L * 16), *rb = (u128 *)calloc(L, 16);
        for (size_t i = 0; i < L; i++) {
            ra[i] = ev[i].a;
            rb[i] = ev[i].b;
        }
        interp_coset_u(ra, L, offset);
        if (K == 2) interp_coset_u(rb, L, offset);
        R.remainder_len = (uint32_t)rl;
        for (size_t k = 0; k < rl; k++) {
            rem[k] = e2_make(ra[k], rb[k]);
            st(R.remainder[k], ra[k]);
        }
        for (size_t k = rl; k < L; k++)
            if (ra[k] || rb[k]) degree_ok = 0;
        e2_hash(rem, rl, K, R.remainder_commitment);
        coin_reseed(&coin, R.remainder_commitment);
        free(ra);
        free(rb);
    }
    if (ev != deep) free(ev);

    /* S7: grinding + query positions [P11] */
    uint64_t nonce = 1;
    for (;; nonce++) {
        uint8_t d[32];
        blake3_merge_with_int(coin.seed, nonce, d);
        uint64_t head;
        memcpy(&head, d, 8);
        unsigned tz = head ? (unsigned)__builtin_ctzll(head) : 64;
        if (tz >= opt->grinding) break;
    }
    R.pow_nonce = nonce;
    {
        uint8_t s2[32];
        blake3_merge_with_int(coin.seed, nonce, s2);
        memcpy(coin.seed, s2, 32);
        coin.counter = 0;
    }
    uint64_t pos[OR_MAX_QUERIES + 1];
    size_t np = 0;
    for (uint32_t q = 0; q < opt->num_queries; q++) {
        uint8_t d[32];
        coin_next(&coin, d);
        uint64_t v;
        memcpy(&v, d, 8);
        pos[np++] = v & (N - 1);
    }
    /* sort_unstable + dedup */
    for (size_t i = 1; i < np; i++)
        for (size_t j = i; j > 0 && pos[j - 1] > pos[j]; j--) {
            uint64_t t = pos[j];
            pos[j] = pos[j - 1];
            pos[j - 1] = t;
        }
    size_t nu = 0;
    for (size_t i = 0; i < np; i++)
        if (nu == 0 || pos[nu - 1] != pos[i]) pos[nu++] = pos[i];
    R.num_positions = (uint32_t)nu;
    memcpy(R.positions, pos, nu * 8);

    /* S8/S9: proof assembly [P13, P14] */
    buf_t pf = {0};
    /* Context */
    bw_u8(&pf, W);
    bw_u8(&pf, 0);
    bw_u8(&pf, 0);
    bw_u8(&pf, (uint8_t)ilog2_sz(n));
    bw_u16(&pf, 0);
    bw_u8(&pf, 16);
    {
        u128 p = F_P;
        bw(&pf, &p, 16);
    }
    bw_u8(&pf, (uint8_t)opt->num_queries);
    bw_u8(&pf, (uint8_t)B);
    bw_u8(&pf, (uint8_t)opt->grinding);
    bw_u8(&pf, (uint8_t)opt->field_extension);
    bw_u8(&pf, (uint8_t)fold);
    bw_u8(&pf, (uint8_t)opt->fri_rem_max_deg);
    bw_u8(&pf, (uint8_t)nu);
    /* Commitments */
    bw_u16(&pf, (uint16_t)(32 * (2 + nl + 1)));
    bw(&pf, R.trace_root, 32);
    bw(&pf, R.constraint_root, 32);
    for (size_t l = 0; l < nl; l++) bw(&pf, R.fri_roots[l], 32);
    bw(&pf, R.remainder_commitment, 32);
    /* trace queries (one segment) */
    {
        buf_t paths = {0};
        prove_batch(leaves, tnodes, N, pos, nu, &paths);
        uint8_t *vals = (uint8_t *)malloc(nu * W * 16);
        for (size_t q = 0; q < nu; q++) memcpy(vals + q * W * 16, lde + pos[q] * W, W * 16);
        bw_u8(&pf, 1);
        write_queries(&pf, vals, nu * W * 16, &paths);
        free(vals);
        free(paths.p);
    }
    /* constraint queries: rows of C E values */
    {
        buf_t paths = {0};
        prove_batch(cleaves, cnodes, N, pos, nu, &paths);
        uint8_t *vals = (uint8_t *)malloc(nu * CK * 16);
        for (size_t q = 0; q < nu; q++) memcpy(vals + q * CK * 16, clde + pos[q] * CK, CK * 16);
        write_queries(&pf, vals, nu * CK * 16, &paths);
        free(vals);
        free(paths.p);
    }
    /* OOD frame: trace states (frame size 2, interleaved per column), constraint evaluations [P7] */
    {
        u128 flat[2 * OR_MAX_CCOLS + 4];
        bw_u16(&pf, (uint16_t)(1 + 2 * W * 16 * K));
        bw_u8(&pf, 2);
        for (int c = 0; c < W; c++) {
            e2_flatten(&ood[c], 1, K, flat);
            bw(&pf, flat, 16 * K);
            e2_flatten(&ood[W + c], 1, K, flat);
            bw(&pf, flat, 16 * K);
        }
        bw_u16(&pf, (uint16_t)(C * 16 * K));
        e2_flatten(oodc, C, K, flat);
        bw(&pf, flat, C * 16 * K);
    }
    /* FRI proof: per layer, fold positions (first-occurrence order), rows + batch proof */
    {
        bw_u8(&pf, (uint8_t)nl);
        uint64_t fp[OR_MAX_QUERIES + 1];
        size_t nfp = nu;
        memcpy(fp, pos, nu * 8);
        size_t dsz = N;
        for (size_t l = 0; l < nl; l++) {
            size_t target = dsz / fold;
            uint64_t nfpv[OR_MAX_QUERIES + 1];
            size_t m = 0;
            for (size_t i = 0; i < nfp; i++) {
                uint64_t p = fp[i] % target;
                int seen = 0;
                for (size_t j = 0; j < m; j++)
                    if (nfpv[j] == p) seen = 1;
                if (!seen) nfpv[m++] = p;
            }
            buf_t paths = {0};
            prove_batch(layer_leaves[l], layer_nodes[l], layer_rows[l], nfpv, m, &paths);
            u128 *vals = (u128 *)malloc(m * fold * K * 16);
            for (size_t q = 0; q < m; q++) e2_flatten(layer_vals[l] + nfpv[q] * fold, fold, K, vals + q * fold * K);
            write_queries(&pf, (const uint8_t *)vals, m * fold * K * 16, &paths);
            free(vals);
            free(paths.p);
            memcpy(fp, nfpv, m * 8);
            nfp = m;
            dsz = target;
        }
        u128 flat[2 * OR_MAX_REMAINDER];
        e2_flatten(rem, rl, K, flat);
        bw_u16(&pf, (uint16_t)(rl * 16 * K));
        bw(&pf, flat, rl * 16 * K);
        bw_u8(&pf, 0); /* num_partitions = 1, stored as log2 */
    }
    bw_u64(&pf, nonce);
    bw_u8(&pf, 0); /* gkr_proof: None */

    /* outputs */
    int rc = degree_ok ? OR_OK : OR_ERR_DEGREE; /* trace violates the AIR: composition degree too high */
    if (rec) *rec = R;
    if (dump) {
        if (dump->trace_polys) memcpy(dump->trace_polys, polys, W * n * 16);
        if (dump->trace_lde) memcpy(dump->trace_lde, lde, N * W * 16);
        if (dump->trace_leaves) memcpy(dump->trace_leaves, leaves, N * 32);
        if (dump->comp_polys) memcpy(dump->comp_polys, cpolys, CK * n * 16);
        if (dump->comp_lde) memcpy(dump->comp_lde, clde, N * CK * 16);
    }
    if (proof_out && *proof_len >= pf.len)
        memcpy(proof_out, pf.p, pf.len);
    else if (rc == OR_OK)
        rc = OR_ERR_BUFFER_TOO_SMALL;
    *proof_len = pf.len;
    free(pf.p);
    for (size_t l = 0; l < nl; l++) {
        free(layer_vals[l]);
        free(layer_leaves[l]);
        free(layer_nodes[l]);
    }
    free(deep);
    free(cpolys);
    free(clde);
    free(cleaves);
    free(cnodes);
    free(comp);
    free(polys);
    free(lde);
    free(leaves);
    free(tnodes);
    return rc;
}
