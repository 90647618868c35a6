/*
 * verifier.c -- oracle: winterfell 0.9 `verify::<ProcessorAir, Blake3_256, DefaultRandomCoin>`
 * (call sites vm/src/lib.rs:93-98, examples/linear_regression/src/main.rs:85) restated for this
 * AIR and the proof layout of prover.c.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * It re-derives the transcript, checks every Merkle batch opening, the out-of-domain identity
 * H(z) = sum_j z^(j*n) H_j(z) against ProcessorAir::evaluate_transition at z, the DEEP values at
 * the query positions, every FRI folding step and the remainder polynomial, and the conjectured
 * security (winter-air ProofOptions): min(128 - log2 N, log2(B) * q [+ grinding]) - 1.
 */
#include <stdio.h>

#include "ext.h"
#include "internal.h"

#define W 28
#define NUM_TCONS 20
#define NUM_ASSERTS 22

typedef struct {
    const uint8_t *p;
    size_t len, off;
    int bad;
} rd_t;
static const uint8_t *rd(rd_t *r, size_t n) {
    if (r->off + n > r->len) {
        r->bad = 1;
        return NULL;
    }
    const uint8_t *q = r->p + r->off;
    r->off += n;
    return q;
}
static uint8_t rd_u8(rd_t *r) {
    const uint8_t *q = rd(r, 1);
    return q ? q[0] : 0;
}
static uint16_t rd_u16(rd_t *r) {
    const uint8_t *q = rd(r, 2);
    return q ? (uint16_t)(q[0] | q[1] << 8) : 0;
}
static uint32_t rd_u32(rd_t *r) {
    const uint8_t *q = rd(r, 4);
    uint32_t v = 0;
    if (q) memcpy(&v, q, 4);
    return v;
}

typedef struct {
    uint8_t seed[32];
    uint64_t counter;
} vcoin_t;
static void vc_reseed(vcoin_t *c, const uint8_t d[32]) {
    uint8_t o[32];
    or_blake3_merge(c->seed, d, o);
    memcpy(c->seed, o, 32);
    c->counter = 0;
}
/* draw::<E> (see coin_draw_e in prover.c) */
static e2 vc_draw(vcoin_t *c, int k) {
    for (int i = 0; i < 1000; i++) {
        uint8_t d[32];
        c->counter++;
        blake3_merge_with_int(c->seed, c->counter, d);
        const u128 a = ld(d), b = k == 2 ? ld(d + 16) : 0;
        if (a < F_P && b < F_P) return e2_make(a, b);
    }
    return e2_base(0);
}
/* n E values of k base components each from bytes; 0 when a component is not canonical */
static int rd_e(const uint8_t *p, size_t n, int k, e2 *out) {
    for (size_t i = 0; i < n; i++) {
        const u128 a = ld(p + 16 * k * i), b = k == 2 ? ld(p + 16 * k * i + 16) : 0;
        if (a >= F_P || b >= F_P) return 0;
        out[i] = e2_make(a, b);
    }
    return 1;
}

#define FAIL(...)                                   \
    do {                                            \
        if (msg) snprintf(msg, msg_cap, __VA_ARGS__); \
        rc = -30;                                   \
        goto out;                                   \
    } while (0)

/* BatchMerkleProof::get_root over the serialized node vectors */
static int batch_root(rd_t *r, const uint8_t *leaf_digests, const uint64_t *idx, size_t k, unsigned depth,
                      uint8_t root[32]) {
    size_t nv = rd_u8(r);
    uint64_t norm[OR_MAX_QUERIES + 1];
    size_t nn = 0;
    for (size_t i = 0; i < k; i++) {
        uint64_t v = idx[i] & ~1ULL;
        int dup = 0;
        for (size_t t = 0; t < nn; t++) dup |= norm[t] == v;
        if (dup) continue;
        size_t j = nn++;
        while (j > 0 && norm[j - 1] > v) {
            norm[j] = norm[j - 1];
            j--;
        }
        norm[j] = v;
    }
    if (nv != nn) return -1;
    const uint8_t *vec[OR_MAX_QUERIES + 1];
    size_t vlen[OR_MAX_QUERIES + 1], ptr[OR_MAX_QUERIES + 1];
    for (size_t i = 0; i < nv; i++) {
        vlen[i] = rd_u8(r);
        vec[i] = rd(r, 32 * vlen[i]);
        if (r->bad) return -1;
    }
    /* map node index -> digest (small linear maps suffice for <= 255 queries) */
    size_t cap = (depth + 2) * (nn + 1) * 2;
    uint64_t *keys = (uint64_t *)malloc(cap * 8);
    uint8_t *vals = (uint8_t *)malloc(cap * 32);
    size_t nkv = 0;
#define PUT(key, d)                              \
    do {                                         \
        keys[nkv] = (key);                       \
        memcpy(vals + 32 * nkv, (d), 32);        \
        nkv++;                                   \
    } while (0)
    uint64_t next[OR_MAX_QUERIES + 1], cur[OR_MAX_QUERIES + 1];
    size_t nnext = 0;
    uint64_t off = 1ULL << depth;
    int rc = 0;
    for (size_t i = 0; i < nn; i++) {
        uint8_t buf[64];
        int have0 = -1, have1 = -1;
        for (size_t t = 0; t < k; t++) {
            if (idx[t] == norm[i]) have0 = (int)t;
            if (idx[t] == norm[i] + 1) have1 = (int)t;
        }
        size_t p = 0;
        if (have0 >= 0) memcpy(buf, leaf_digests + 32 * have0, 32);
        else {
            if (vlen[i] < 1) { rc = -1; goto done; }
            memcpy(buf, vec[i], 32);
            p = 1;
        }
        if (have1 >= 0) memcpy(buf + 32, leaf_digests + 32 * have1, 32);
        else {
            if (have0 < 0 || vlen[i] < 1) { rc = -1; goto done; }
            memcpy(buf + 32, vec[i], 32);
            p = 1;
        }
        ptr[i] = p;
        uint8_t par[32];
        or_blake3(buf, 64, par);
        PUT((off + norm[i]) >> 1, par);
        next[nnext++] = (off + norm[i]) >> 1;
    }
    for (unsigned lvl = 1; lvl < depth; lvl++) {
        memcpy(cur, next, nnext * 8);
        size_t ncur = nnext;
        nnext = 0;
        for (size_t i = 0; i < ncur; i++) {
            uint64_t node = cur[i], sib = node ^ 1;
            const uint8_t *sd = NULL, *nd = NULL;
            if (i + 1 < ncur && cur[i + 1] == sib) {
                for (size_t t = 0; t < nkv; t++)
                    if (keys[t] == sib) sd = vals + 32 * t;
                i++;
            } else {
                if (ptr[i] >= vlen[i]) { rc = -1; goto done; }
                sd = vec[i] + 32 * ptr[i]++;
            }
            for (size_t t = 0; t < nkv; t++)
                if (keys[t] == node) nd = vals + 32 * t;
            if (!sd || !nd) { rc = -1; goto done; }
            uint8_t buf[64], par[32];
            if (node & 1) {
                memcpy(buf, sd, 32);
                memcpy(buf + 32, nd, 32);
            } else {
                memcpy(buf, nd, 32);
                memcpy(buf + 32, sd, 32);
            }
            or_blake3(buf, 64, par);
            PUT(node >> 1, par);
            next[nnext++] = node >> 1;
        }
    }
    rc = -1;
    for (size_t t = 0; t < nkv; t++)
        if (keys[t] == 1) {
            memcpy(root, vals + 32 * t, 32);
            rc = 0;
        }
done:
#undef PUT
    free(keys);
    free(vals);
    return rc;
}

int or_verify(const uint8_t *proof, size_t proof_len, const or_pub_inputs *pub, uint32_t min_security, char *msg,
              size_t msg_cap) {
    int rc = 0;
    rd_t r = {proof, proof_len, 0, 0};
    uint64_t pos[OR_MAX_QUERIES + 1], fp[OR_MAX_QUERIES + 1];
    u128 *tvals = NULL, *cvals = NULL;
    e2 evals[OR_MAX_QUERIES + 1];
    /* ---- context */
    uint8_t width = rd_u8(&r), auxw = rd_u8(&r), auxr = rd_u8(&r), logn = rd_u8(&r);
    uint16_t meta = rd_u16(&r);
    rd(&r, meta);
    uint8_t mlen = rd_u8(&r);
    const uint8_t *mod = rd(&r, mlen);
    uint8_t nq = rd_u8(&r), B = rd_u8(&r), grind = rd_u8(&r), ext = rd_u8(&r), fold = rd_u8(&r),
            remdeg = rd_u8(&r);
    uint8_t nu = rd_u8(&r);
    if (r.bad || width != W || auxw || auxr || mlen != 16 || (ext != 1 && ext != 2) || logn < 4 || logn > 32 || B < 8 ||
        (B & (B - 1)) || !(fold == 2 || fold == 4 || fold == 8 || fold == 16))
        FAIL("malformed proof context");
    {
        u128 p = F_P;
        if (memcmp(mod, &p, 16)) FAIL("field modulus mismatch");
    }
    const size_t n = (size_t)1 << logn, N = n * B;
    const int K = ext;
    /* conjectured security */
    {
        unsigned logN = logn + ilog2_sz(B);
        int field_sec = 128 * K - (int)logN;
        int q_sec = (int)ilog2_sz(B) * nq;
        if (q_sec >= 80) q_sec += grind;
        int sec = (field_sec < q_sec ? field_sec : q_sec) - 1;
        if (sec > 128) sec = 128;
        if (sec < (int)min_security) FAIL("insufficient proof security: %d < %u", sec, min_security);
    }
    size_t nl = 0, max_rem = (size_t)(remdeg + 1) * B;
    for (size_t s = N; s > max_rem; s /= fold) nl++;
    /* ---- commitments */
    uint16_t clen = rd_u16(&r);
    const uint8_t *coms = rd(&r, clen);
    if (r.bad || clen != 32 * (2 + nl + 1)) FAIL("malformed commitments");
    /* ---- transcript up to the queries */
    vcoin_t coin;
    {
        u128 e[26];
        size_t k = 0;
        e[k++] = (u128)W << 16;
        e[k++] = n;
        e[k++] = (u128)(uint64_t)F_P;
        e[k++] = (u128)(uint64_t)(F_P >> 64);
        e[k++] = ((u128)ext << 16) | ((u128)fold << 8) | remdeg;
        e[k++] = grind;
        e[k++] = B;
        e[k++] = nq;
        for (int i = 0; i < 2; i++) e[k++] = ld(pub->program_hash[i]);
        for (int i = 0; i < 16; i++) e[k++] = ld(pub->stack_outputs[i]);
        blake3_hash_elems(e, k, coin.seed);
        coin.counter = 0;
    }
    vc_reseed(&coin, coms);
    e2 ct[NUM_TCONS], cb[NUM_ASSERTS];
    for (int i = 0; i < NUM_TCONS; i++) ct[i] = vc_draw(&coin, K);
    for (int i = 0; i < NUM_ASSERTS; i++) cb[i] = vc_draw(&coin, K);
    vc_reseed(&coin, coms + 32);
    const e2 z = vc_draw(&coin, K);
    /* ---- read the remaining sections in proof order */
    uint8_t nseg = rd_u8(&r);
    if (nseg != 1) FAIL("expected one trace segment");
    uint32_t tvl = rd_u32(&r);
    const uint8_t *tv = rd(&r, tvl);
    uint32_t tpl = rd_u32(&r);
    const uint8_t *tp = rd(&r, tpl);
    uint32_t cvl = rd_u32(&r);
    const uint8_t *cv = rd(&r, cvl);
    uint32_t cpl = rd_u32(&r);
    const uint8_t *cp = rd(&r, cpl);
    uint16_t tsl = rd_u16(&r);
    const uint8_t *ts = rd(&r, tsl);
    uint16_t oel = rd_u16(&r);
    const uint8_t *oe = rd(&r, oel);
    if (r.bad || tsl != 1 + 2 * W * 16 * K || ts[0] != 2 || oel % (16 * K) || oel / (16 * K) > OR_MAX_CCOLS ||
        oel == 0 || (size_t)(oel / (16 * K)) != (size_t)or_num_comp_cols((size_t)1 << logn))
        FAIL("malformed OOD frame");
    const size_t C = oel / (16 * K);
    e2 oz[W], ozg[W], oc[OR_MAX_CCOLS];
    for (int c = 0; c < W; c++)
        if (!rd_e(ts + 1 + 32 * K * c, 1, K, &oz[c]) || !rd_e(ts + 1 + 32 * K * c + 16 * K, 1, K, &ozg[c]))
            FAIL("non-canonical OOD value");
    if (!rd_e(oe, C, K, oc)) FAIL("non-canonical OOD value");
    {
        e2 both[2 * W];
        memcpy(both, oz, sizeof oz);
        memcpy(both + W, ozg, sizeof ozg);
        uint8_t h[32];
        e2_hash(both, 2 * W, K, h);
        vc_reseed(&coin, h);
        e2_hash(oc, C, K, h);
        vc_reseed(&coin, h);
    }
    /* ---- OOD consistency: H(z) from the AIR at z vs sum_j z^(jn) H_j(z) */
    {
        const u128 g = f_root_of_unity(logn);
        e2 per[9], ev[NUM_TCONS];
        u128 pc[9][16];
        for (unsigned s = 0; s < 16; s++) {
            u128 row[9];
            air_periodic_u(s, row);
            for (int j = 0; j < 9; j++) pc[j][s] = row[j];
        }
        const e2 zp = e2_exp(z, n / 16);
        for (int j = 0; j < 9; j++) {
            interp_coset_u(pc[j], 16, 1);
            per[j] = poly_eval_e(pc[j], 16, zp);
        }
        air_eval_e(oz, ozg, per, pub->lwe_size, pub->delta, ev);
        e2 t = e2_base(0);
        for (int k = 0; k < NUM_TCONS; k++) t = e2_add(t, e2_mul(ct[k], ev[k]));
        const e2 gl2 = e2_base(f_exp(g, n - 2)), gl1 = e2_base(f_exp(g, n - 1)), one = e2_base(1);
        const e2 zn = e2_exp(z, n);
        e2 h = e2_mul(e2_mul(t, e2_mul(e2_sub(z, gl2), e2_sub(z, gl1))), e2_inv(e2_sub(zn, one)));
        const int fc[12] = {0, 7, 8, 11, 12, 13, 14, 15, 16, 17, 18, 19};
        e2 b0 = e2_base(0), b1 = e2_base(0);
        for (int i = 0; i < 12; i++) b0 = e2_add(b0, e2_mul(cb[i], oz[fc[i]]));
        for (int i = 0; i < 2; i++)
            b1 = e2_add(b1, e2_mul(cb[12 + i], e2_sub(oz[7 + i], e2_base(ld(pub->program_hash[i])))));
        for (int i = 0; i < 8; i++)
            b1 = e2_add(b1, e2_mul(cb[14 + i], e2_sub(oz[12 + i], e2_base(ld(pub->stack_outputs[i])))));
        h = e2_add(h, e2_mul(b0, e2_inv(e2_sub(z, one))));
        h = e2_add(h, e2_mul(b1, e2_inv(e2_sub(z, gl2))));
        /* H(z) = sum_j z^(jn) H_j(z); with k = 2, H_j(z) = oc[j] as the E-valued column */
        e2 hc = e2_base(0), zz = one;
        for (size_t j = 0; j < C; j++) {
            hc = e2_add(hc, e2_mul(zz, oc[j]));
            zz = e2_mul(zz, zn);
        }
        if (!e2_eq(h, hc)) FAIL("out-of-domain constraint evaluation mismatch");
    }
    e2 at[W], ac[OR_MAX_CCOLS];
    for (int c = 0; c < W; c++) at[c] = vc_draw(&coin, K);
    for (size_t j = 0; j < C; j++) ac[j] = vc_draw(&coin, K);
    e2 alphas[OR_MAX_FRI_LAYERS];
    for (size_t l = 0; l < nl; l++) {
        vc_reseed(&coin, coms + 64 + 32 * l);
        alphas[l] = vc_draw(&coin, K);
    }
    vc_reseed(&coin, coms + 64 + 32 * nl);
    /* ---- FRI section (parsed now, checked after the queries) */
    uint8_t fnl = rd_u8(&r);
    if (fnl != nl) FAIL("wrong number of FRI layers");
    const uint8_t *lv[OR_MAX_FRI_LAYERS], *lp[OR_MAX_FRI_LAYERS];
    uint32_t lvl[OR_MAX_FRI_LAYERS], lpl[OR_MAX_FRI_LAYERS];
    for (size_t l = 0; l < nl; l++) {
        lvl[l] = rd_u32(&r);
        lv[l] = rd(&r, lvl[l]);
        lpl[l] = rd_u32(&r);
        lp[l] = rd(&r, lpl[l]);
    }
    uint16_t rml = rd_u16(&r);
    const uint8_t *rm = rd(&r, rml);
    uint8_t nparts = rd_u8(&r);
    const uint8_t *nonce_b = rd(&r, 8);
    uint8_t gkr = rd_u8(&r);
    if (r.bad || nparts != 0 || gkr != 0 || r.off != r.len) FAIL("malformed proof tail");
    const size_t rem_len = rml / (16 * K);
    {
        uint8_t h[32];
        or_blake3(rm, rml, h);
        if (memcmp(h, coms + 64 + 32 * nl, 32)) FAIL("remainder commitment mismatch");
    }
    /* ---- grinding and query positions */
    uint64_t nonce;
    memcpy(&nonce, nonce_b, 8);
    {
        uint8_t d[32];
        blake3_merge_with_int(coin.seed, nonce, d);
        uint64_t head;
        memcpy(&head, d, 8);
        unsigned tz = head ? (unsigned)__builtin_ctzll(head) : 64;
        if (tz < grind) FAIL("query seed proof-of-work is invalid");
        memcpy(coin.seed, d, 32);
        coin.counter = 0;
    }
    size_t np = 0;
    for (uint32_t q = 0; q < nq; q++) {
        uint8_t d[32];
        coin.counter++;
        blake3_merge_with_int(coin.seed, coin.counter, d);
        uint64_t v;
        memcpy(&v, d, 8);
        pos[np++] = v & (N - 1);
    }
    for (size_t i = 1; i < np; i++)
        for (size_t j = i; j > 0 && pos[j - 1] > pos[j]; j--) {
            uint64_t t = pos[j];
            pos[j] = pos[j - 1];
            pos[j - 1] = t;
        }
    size_t nuq = 0;
    for (size_t i = 0; i < np; i++)
        if (nuq == 0 || pos[nuq - 1] != pos[i]) pos[nuq++] = pos[i];
    if (nuq != nu) FAIL("number of unique queries mismatch");
    /* ---- trace and constraint openings */
    const size_t CK = C * K;
    if (tvl != nu * W * 16 || cvl != nu * CK * 16) FAIL("malformed query values");
    tvals = (u128 *)malloc(nu * W * 16);
    cvals = (u128 *)malloc(nu * CK * 16);
    memcpy(tvals, tv, tvl);
    memcpy(cvals, cv, cvl);
    {
        uint8_t *dig = (uint8_t *)malloc(nu * 32), root[32];
        for (size_t q = 0; q < nu; q++) blake3_hash_elems(tvals + q * W, W, dig + 32 * q);
        rd_t pr = {tp, tpl, 0, 0};
        int e = batch_root(&pr, dig, pos, nu, logn + ilog2_sz(B), root);
        if (e || pr.off != pr.len || memcmp(root, coms, 32)) {
            free(dig);
            FAIL("trace query does not match the commitment");
        }
        for (size_t q = 0; q < nu; q++) blake3_hash_elems(cvals + q * CK, CK, dig + 32 * q);
        rd_t pc2 = {cp, cpl, 0, 0};
        e = batch_root(&pc2, dig, pos, nu, logn + ilog2_sz(B), root);
        free(dig);
        if (e || pc2.off != pc2.len || memcmp(root, coms + 32, 32)) FAIL("constraint query does not match the commitment");
    }
    /* ---- DEEP values at the query positions (in E) */
    {
        const u128 wN = f_root_of_unity(logn + ilog2_sz(B));
        const e2 zg = e2_mulb(z, f_root_of_unity(logn));
        for (size_t q = 0; q < nu; q++) {
            const e2 x = e2_base(f_mul(F_GENERATOR, f_exp(wN, pos[q])));
            e2 s1 = e2_base(0), s2 = e2_base(0), hv[OR_MAX_CCOLS];
            for (int c = 0; c < W; c++) {
                const e2 v = e2_base(tvals[q * W + c]);
                s1 = e2_add(s1, e2_mul(at[c], e2_sub(v, oz[c])));
                s2 = e2_add(s2, e2_mul(at[c], e2_sub(v, ozg[c])));
            }
            if (!rd_e((const uint8_t *)(cvals + q * CK), C, K, hv)) FAIL("non-canonical constraint value");
            for (size_t j = 0; j < C; j++) s1 = e2_add(s1, e2_mul(ac[j], e2_sub(hv[j], oc[j])));
            evals[q] = e2_add(e2_mul(s1, e2_inv(e2_sub(x, z))), e2_mul(s2, e2_inv(e2_sub(x, zg))));
        }
    }
    /* ---- FRI layers */
    {
        size_t dsz = N, ncur = nu;
        memcpy(fp, pos, nu * 8);
        u128 dgen = f_root_of_unity(ilog2_sz(N));
        for (size_t l = 0; l < nl; l++) {
            size_t target = dsz / fold;
            uint64_t folded[OR_MAX_QUERIES + 1];
            size_t m = 0;
            for (size_t i = 0; i < ncur; i++) {
                uint64_t p = fp[i] % target;
                int seen = 0;
                for (size_t j = 0; j < m; j++) seen |= folded[j] == p;
                if (!seen) folded[m++] = p;
            }
            if (lvl[l] != m * fold * 16 * K) FAIL("malformed FRI layer %zu", l);
            e2 *rows = (e2 *)malloc(m * fold * sizeof(e2));
            if (!rd_e(lv[l], m * fold, K, rows)) {
                free(rows);
                FAIL("non-canonical FRI value in layer %zu", l);
            }
            uint8_t *dig = (uint8_t *)malloc(m * 32), root[32];
            for (size_t q = 0; q < m; q++) blake3_hash_elems((const u128 *)(lv[l] + 16 * K * fold * q), fold * K, dig + 32 * q);
            rd_t pr = {lp[l], lpl[l], 0, 0};
            int e = batch_root(&pr, dig, folded, m, ilog2_sz(target), root);
            free(dig);
            if (e || pr.off != pr.len || memcmp(root, coms + 64 + 32 * l, 32)) {
                free(rows);
                FAIL("FRI layer %zu query does not match the commitment", l);
            }
            /* get_query_values: position p sits in row (p % target), column (p / target) */
            for (size_t i = 0; i < ncur; i++) {
                size_t ri = 0;
                while (folded[ri] != fp[i] % target) ri++;
                if (!e2_eq(rows[ri * fold + fp[i] / target], evals[i])) {
                    free(rows);
                    FAIL("FRI layer %zu folding mismatch", l);
                }
            }
            e2 nxt[OR_MAX_QUERIES + 1];
            for (size_t q = 0; q < m; q++) {
                u128 xe = f_mul(f_exp(dgen, folded[q]), F_GENERATOR), va[16], vb[16];
                for (size_t t = 0; t < fold; t++) {
                    va[t] = rows[q * fold + t].a;
                    vb[t] = rows[q * fold + t].b;
                }
                interp_coset_u(va, fold, xe);
                if (K == 2) interp_coset_u(vb, fold, xe);
                e2 acc = e2_base(0);
                for (size_t t = fold; t-- > 0;) acc = e2_add(e2_mul(acc, alphas[l]), e2_make(va[t], K == 2 ? vb[t] : 0));
                nxt[q] = acc;
            }
            free(rows);
            memcpy(evals, nxt, m * sizeof(e2));
            memcpy(fp, folded, m * 8);
            ncur = m;
            dgen = f_exp(dgen, fold);
            dsz = target;
        }
        /* remainder: an E polynomial with rem_len coefficients, evaluated at base points */
        if (rem_len != dsz / B || rml != rem_len * 16 * K) FAIL("remainder has wrong size");
        e2 *rp = (e2 *)malloc((rem_len + 1) * sizeof(e2));
        if (!rd_e(rm, rem_len, K, rp)) {
            free(rp);
            FAIL("non-canonical remainder coefficient");
        }
        for (size_t i = 0; i < ncur; i++) {
            const e2 x = e2_base(f_mul(F_GENERATOR, f_exp(dgen, fp[i])));
            e2 acc = e2_base(0);
            for (size_t t = rem_len; t-- > 0;) acc = e2_add(e2_mul(acc, x), rp[t]);
            if (!e2_eq(acc, evals[i])) {
                free(rp);
                FAIL("FRI remainder mismatch");
            }
        }
        free(rp);
    }
    if (msg) msg[0] = 0;
out:
    free(tvals);
    free(cvals);
    return rc;
}
