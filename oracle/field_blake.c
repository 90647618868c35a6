/*
 * field_blake.c -- oracle: f128 field API, radix-2 NTT, BLAKE3-256 and binary Merkle trees.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * f128: winter-math `fields::f128::BaseElement` as used by prover/src/lib.rs:4 (third-party
 *   winter-math 0.9.x, not vendored; Cargo.lock:538-633).  Canonical, 16-byte LE.
 * NTT: evaluation / interpolation over cosets offset*<w_N> in natural order -- the semantics of
 *   winter-math `fft::evaluate_poly_with_offset` / `interpolate_poly_with_offset`.
 * BLAKE3: the public BLAKE3 specification (blake3 1.5.4, Cargo.lock:48), hash mode, 32-byte out.
 *   winter-crypto `Blake3_256::hash_elements` hashes the canonical LE element bytes, `merge`
 *   hashes the 64-byte concatenation, `merge_with_int` hashes seed(32) || u64 LE (40 bytes).
 * Merkle: winter-crypto `MerkleTree::new`: nodes[n + i] = merge(leaf[2i], leaf[2i+1]),
 *   nodes[i] = merge(nodes[2i], nodes[2i+1]), root = nodes[1].
 */
#include "internal.h"

/* ------------------------------------------------------------------ field API */
void or_fadd(const void *a, const void *b, void *out) { st(out, f_add(ld(a), ld(b))); }
void or_fsub(const void *a, const void *b, void *out) { st(out, f_sub(ld(a), ld(b))); }
void or_fmul(const void *a, const void *b, void *out) { st(out, f_mul(ld(a), ld(b))); }
void or_finv(const void *a, void *out) { st(out, f_inv(ld(a))); }
void or_fexp(const void *a, const void *e, void *out) { st(out, f_exp(ld(a), ld(e))); }
void or_root_of_unity(uint32_t log_n, void *out) { st(out, f_root_of_unity(log_n)); }

/* ------------------------------------------------------------------ NTT */
/* A[j] = sum_k a[k] w^(jk), natural order in and out (iterative Cooley-Tukey). */
void ntt_natural(u128 *a, size_t n, u128 w) {
    unsigned lg = ilog2_sz(n);
    for (size_t i = 0; i < n; i++) {
        size_t r = 0;
        for (unsigned b = 0; b < lg; b++) r |= ((i >> b) & 1) << (lg - 1 - b);
        if (i < r) {
            u128 t = a[i];
            a[i] = a[r];
            a[r] = t;
        }
    }
    for (size_t len = 2; len <= n; len <<= 1) {
        u128 wl = f_exp(w, (u128)(n / len));
        size_t half = len >> 1;
        u128 *tw = (u128 *)malloc(half * sizeof(u128));
        tw[0] = 1;
        for (size_t j = 1; j < half; j++) tw[j] = f_mul(tw[j - 1], wl);
        for (size_t i = 0; i < n; i += len) {
            for (size_t j = 0; j < half; j++) {
                u128 u = a[i + j], v = f_mul(a[i + j + half], tw[j]);
                a[i + j] = f_add(u, v);
                a[i + j + half] = f_sub(u, v);
            }
        }
        free(tw);
    }
}

void eval_coset_u(const u128 *coeffs, size_t m, size_t size, u128 offset, u128 *out) {
    u128 s = 1;
    for (size_t k = 0; k < size; k++) {
        out[k] = k < m ? f_mul(coeffs[k], s) : 0;
        s = f_mul(s, offset);
    }
    ntt_natural(out, size, f_root_of_unity(ilog2_sz(size)));
}

void interp_coset_u(u128 *vals, size_t size, u128 offset) {
    ntt_natural(vals, size, f_inv(f_root_of_unity(ilog2_sz(size))));
    u128 inv_n = f_inv((u128)size), inv_off = f_inv(offset), s = inv_n;
    for (size_t k = 0; k < size; k++) {
        vals[k] = f_mul(vals[k], s);
        s = f_mul(s, inv_off);
    }
}

u128 poly_eval(const u128 *c, size_t m, u128 x) {
    u128 r = 0;
    for (size_t k = m; k-- > 0;) r = f_add(f_mul(r, x), c[k]);
    return r;
}

int or_eval_coset(const void *coeffs, size_t m, size_t size, const void *offset, void *out) {
    if (size == 0 || (size & (size - 1)) || m > size) return OR_ERR_INVALID_ARG;
    u128 *c = (u128 *)malloc(m * 16 + 16), *o = (u128 *)malloc(size * 16);
    memcpy(c, coeffs, m * 16);
    eval_coset_u(c, m, size, ld(offset), o);
    memcpy(out, o, size * 16);
    free(c);
    free(o);
    return OR_OK;
}

int or_interp_coset(void *vals, size_t size, const void *offset) {
    if (size == 0 || (size & (size - 1))) return OR_ERR_INVALID_ARG;
    u128 *v = (u128 *)malloc(size * 16);
    memcpy(v, vals, size * 16);
    interp_coset_u(v, size, ld(offset));
    memcpy(vals, v, size * 16);
    free(v);
    return OR_OK;
}

/* ------------------------------------------------------------------ BLAKE3 */
static const uint32_t B3_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                  0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const unsigned B3_PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

static inline uint32_t rotr(uint32_t x, unsigned n) { return (x >> n) | (x << (32 - n)); }

static void g(uint32_t *s, int a, int b, int c, int d, uint32_t mx, uint32_t my) {
    s[a] = s[a] + s[b] + mx;
    s[d] = rotr(s[d] ^ s[a], 16);
    s[c] = s[c] + s[d];
    s[b] = rotr(s[b] ^ s[c], 12);
    s[a] = s[a] + s[b] + my;
    s[d] = rotr(s[d] ^ s[a], 8);
    s[c] = s[c] + s[d];
    s[b] = rotr(s[b] ^ s[c], 7);
}

static void compress(const uint32_t cv[8], const uint8_t block[64], uint64_t counter, uint32_t block_len,
                     uint32_t flags, uint32_t out[8]) {
    uint32_t m[16], s[16], t[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)block[4 * i] | ((uint32_t)block[4 * i + 1] << 8) | ((uint32_t)block[4 * i + 2] << 16) |
               ((uint32_t)block[4 * i + 3] << 24);
    for (int i = 0; i < 8; i++) s[i] = cv[i];
    for (int i = 0; i < 4; i++) s[8 + i] = B3_IV[i];
    s[12] = (uint32_t)counter;
    s[13] = (uint32_t)(counter >> 32);
    s[14] = block_len;
    s[15] = flags;
    for (int r = 0; r < 7; r++) {
        g(s, 0, 4, 8, 12, m[0], m[1]);
        g(s, 1, 5, 9, 13, m[2], m[3]);
        g(s, 2, 6, 10, 14, m[4], m[5]);
        g(s, 3, 7, 11, 15, m[6], m[7]);
        g(s, 0, 5, 10, 15, m[8], m[9]);
        g(s, 1, 6, 11, 12, m[10], m[11]);
        g(s, 2, 7, 8, 13, m[12], m[13]);
        g(s, 3, 4, 9, 14, m[14], m[15]);
        if (r < 6) {
            for (int i = 0; i < 16; i++) t[i] = m[B3_PERM[i]];
            memcpy(m, t, sizeof m);
        }
    }
    for (int i = 0; i < 8; i++) out[i] = s[i] ^ s[i + 8];
}

/* chaining value of one chunk (<= 1024 bytes); `root` sets ROOT on the last block */
static void chunk_cv(const uint8_t *in, size_t len, uint64_t chunk_idx, int root, uint32_t out[8]) {
    uint32_t cv[8];
    memcpy(cv, B3_IV, sizeof cv);
    size_t nblocks = len == 0 ? 1 : (len + 63) / 64;
    for (size_t b = 0; b < nblocks; b++) {
        uint8_t block[64] = {0};
        size_t off = b * 64, bl = len - off < 64 ? len - off : 64;
        if (len) memcpy(block, in + off, bl);
        uint32_t flags = 0;
        if (b == 0) flags |= CHUNK_START;
        if (b == nblocks - 1) flags |= CHUNK_END | (root ? ROOT : 0);
        compress(cv, block, chunk_idx, (uint32_t)(len ? bl : 0), flags, cv);
    }
    memcpy(out, cv, sizeof cv);
}

static void parent_cv(const uint32_t l[8], const uint32_t r[8], int root, uint32_t out[8]) {
    uint8_t block[64];
    for (int i = 0; i < 8; i++)
        for (int k = 0; k < 4; k++) {
            block[4 * i + k] = (uint8_t)(l[i] >> (8 * k));
            block[32 + 4 * i + k] = (uint8_t)(r[i] >> (8 * k));
        }
    compress(B3_IV, block, 0, 64, PARENT | (root ? ROOT : 0), out);
}

/* BLAKE3 tree: the left subtree holds the largest power-of-two number of chunks that still
 * leaves at least one chunk for the right subtree. */
static void subtree_cv(const uint8_t *in, size_t len, uint64_t first_chunk, int root, uint32_t out[8]) {
    if (len <= 1024) {
        chunk_cv(in, len, first_chunk, root, out);
        return;
    }
    size_t chunks = (len + 1023) / 1024, left = 1;
    while (left * 2 < chunks) left *= 2;
    uint32_t lcv[8], rcv[8];
    subtree_cv(in, left * 1024, first_chunk, 0, lcv);
    subtree_cv(in + left * 1024, len - left * 1024, first_chunk + left, 0, rcv);
    parent_cv(lcv, rcv, root, out);
}

void or_blake3(const uint8_t *in, size_t len, uint8_t out[32]) {
    uint32_t h[8];
    subtree_cv(in, len, 0, 1, h);
    for (int i = 0; i < 8; i++)
        for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(h[i] >> (8 * k));
}

void or_blake3_merge(const uint8_t l[32], const uint8_t r[32], uint8_t out[32]) {
    uint8_t buf[64];
    memcpy(buf, l, 32);
    memcpy(buf + 32, r, 32);
    or_blake3(buf, 64, out);
}

void blake3_hash_elems(const u128 *e, size_t k, uint8_t out[32]) {
    /* canonical f128 => raw LE bytes (winter-crypto Blake3_256::hash_elements) */
    or_blake3((const uint8_t *)e, k * 16, out);
}

void blake3_merge_with_int(const uint8_t seed[32], uint64_t v, uint8_t out[32]) {
    uint8_t buf[40];
    memcpy(buf, seed, 32);
    for (int i = 0; i < 8; i++) buf[32 + i] = (uint8_t)(v >> (8 * i));
    or_blake3(buf, 40, out);
}

uint8_t *merkle_build(const uint8_t *leaves, size_t nl) {
    uint8_t *nodes = (uint8_t *)calloc(2 * nl, 32);
    for (size_t i = 0; i < nl / 2; i++) or_blake3_merge(leaves + 64 * i, leaves + 64 * i + 32, nodes + 32 * (nl / 2 + i));
    for (size_t i = nl / 2; i-- > 1;) or_blake3_merge(nodes + 64 * i, nodes + 64 * i + 32, nodes + 32 * i);
    return nodes;
}

void or_merkle_root(const uint8_t *leaves, size_t nl, uint8_t root[32]) {
    uint8_t *nodes = merkle_build(leaves, nl);
    memcpy(root, nodes + 32, 32);
    free(nodes);
}
