// blake3.hpp -- BLAKE3-256 for the prove path (blake3 1.5.4, Cargo.lock:48; used through
// winter-crypto `Blake3_256<f128>`, prover/src/lib.rs:13).
//
// Device side: one compression function plus single-chunk hashing of <= 1024-byte inputs, which
// covers every hash on the GPU path -- trace rows (28 x 16 B = 448 B, 7 blocks), composition rows
// (7 x 16 B = 112 B), FRI rows (8 x 16 B = 128 B) and Merkle merges (64 B).
// Host side: full tree hashing of arbitrary length (the transcript hashes up to a few KiB).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "f128.hpp"

namespace b3 {

static constexpr uint32_t IV0 = 0x6A09E667u, IV1 = 0xBB67AE85u, IV2 = 0x3C6EF372u, IV3 = 0xA54FF53Au,
                          IV4 = 0x510E527Fu, IV5 = 0x9B05688Cu, IV6 = 0x1F83D9ABu, IV7 = 0x5BE0CD19u;
enum : uint32_t { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

ZK_HD uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

#define ZK_B3_G(a, b, c, d, mx, my) \
    do {                            \
        a = a + b + (mx);           \
        d = rotr(d ^ a, 16);        \
        c = c + d;                  \
        b = rotr(b ^ c, 12);        \
        a = a + b + (my);           \
        d = rotr(d ^ a, 8);         \
        c = c + d;                  \
        b = rotr(b ^ c, 7);         \
    } while (0)

// One compression.  cv[8] is updated in place with the first 8 output words.  The message
// schedule is applied by renaming (the permutation is fixed), so no data moves between rounds.
ZK_HD void compress(uint32_t cv[8], const uint32_t m_in[16], uint32_t counter_lo, uint32_t counter_hi,
                    uint32_t block_len, uint32_t flags) {
    uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3], v4 = cv[4], v5 = cv[5], v6 = cv[6], v7 = cv[7];
    uint32_t v8 = IV0, v9 = IV1, v10 = IV2, v11 = IV3, v12 = counter_lo, v13 = counter_hi, v14 = block_len,
             v15 = flags;
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = m_in[i];
#pragma unroll
    for (int r = 0; r < 7; r++) {
        ZK_B3_G(v0, v4, v8, v12, m[0], m[1]);
        ZK_B3_G(v1, v5, v9, v13, m[2], m[3]);
        ZK_B3_G(v2, v6, v10, v14, m[4], m[5]);
        ZK_B3_G(v3, v7, v11, v15, m[6], m[7]);
        ZK_B3_G(v0, v5, v10, v15, m[8], m[9]);
        ZK_B3_G(v1, v6, v11, v12, m[10], m[11]);
        ZK_B3_G(v2, v7, v8, v13, m[12], m[13]);
        ZK_B3_G(v3, v4, v9, v14, m[14], m[15]);
        if (r < 6) {
            // MSG_PERMUTATION = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]
            uint32_t t[16] = {m[2], m[6], m[3], m[10], m[7], m[0], m[4], m[13],
                              m[1], m[11], m[12], m[5], m[9], m[14], m[15], m[8]};
#pragma unroll
            for (int i = 0; i < 16; i++) m[i] = t[i];
        }
    }
    cv[0] = v0 ^ v8;
    cv[1] = v1 ^ v9;
    cv[2] = v2 ^ v10;
    cv[3] = v3 ^ v11;
    cv[4] = v4 ^ v12;
    cv[5] = v5 ^ v13;
    cv[6] = v6 ^ v14;
    cv[7] = v7 ^ v15;
}

ZK_HD void iv(uint32_t cv[8]) {
    cv[0] = IV0; cv[1] = IV1; cv[2] = IV2; cv[3] = IV3;
    cv[4] = IV4; cv[5] = IV5; cv[6] = IV6; cv[7] = IV7;
}

// hash k field elements (16k <= 1024 bytes) given as an element accessor; out = 8 LE words
template <typename Get>
ZK_HD void hash_elements(int k, Get get, uint32_t out[8]) {
    iv(out);
    const int bytes = 16 * k;
    const int nblocks = (bytes + 63) / 64;
    for (int b = 0; b < nblocks; b++) {
        uint32_t m[16];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            int idx = 4 * b + e;
            fe v = idx < k ? get(idx) : fe_zero();
            m[4 * e + 0] = (uint32_t)v.lo;
            m[4 * e + 1] = (uint32_t)(v.lo >> 32);
            m[4 * e + 2] = (uint32_t)v.hi;
            m[4 * e + 3] = (uint32_t)(v.hi >> 32);
        }
        uint32_t len = (uint32_t)(bytes - 64 * b < 64 ? bytes - 64 * b : 64);
        uint32_t flags = (b == 0 ? CHUNK_START : 0) | (b == nblocks - 1 ? (CHUNK_END | ROOT) : 0);
        compress(out, m, 0, 0, len, flags);
    }
}

// merge(left, right) = BLAKE3(left || right) (winter-crypto Blake3_256::merge)
ZK_HD void merge(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        m[i] = l[i];
        m[8 + i] = r[i];
    }
    iv(out);
    compress(out, m, 0, 0, 64, CHUNK_START | CHUNK_END | ROOT);
}

// ------------------------------------------------------------- host: arbitrary-length hashing
__host__ static inline void words_from_bytes(const uint8_t *p, uint32_t *w, int n) {
    for (int i = 0; i < n; i++) w[i] = (uint32_t)p[4 * i] | (uint32_t)p[4 * i + 1] << 8 | (uint32_t)p[4 * i + 2] << 16 | (uint32_t)p[4 * i + 3] << 24;
}
__host__ static inline void chunk_cv(const uint8_t *in, size_t len, uint64_t idx, bool root, uint32_t out[8]) {
    iv(out);
    size_t nb = len == 0 ? 1 : (len + 63) / 64;
    for (size_t b = 0; b < nb; b++) {
        uint8_t blk[64] = {0};
        size_t bl = len - 64 * b < 64 ? len - 64 * b : 64;
        if (len) memcpy(blk, in + 64 * b, bl);
        uint32_t m[16];
        words_from_bytes(blk, m, 16);
        uint32_t flags = (b == 0 ? CHUNK_START : 0) | (b == nb - 1 ? (CHUNK_END | (root ? ROOT : 0)) : 0);
        compress(out, m, (uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)(len ? bl : 0), flags);
    }
}
__host__ static inline void subtree(const uint8_t *in, size_t len, uint64_t first, bool root, uint32_t out[8]) {
    if (len <= 1024) {
        chunk_cv(in, len, first, root, out);
        return;
    }
    size_t chunks = (len + 1023) / 1024, left = 1;
    while (left * 2 < chunks) left *= 2;
    uint32_t l[8], r[8], m[16];
    subtree(in, left * 1024, first, false, l);
    subtree(in + left * 1024, len - left * 1024, first + left, false, r);
    for (int i = 0; i < 8; i++) {
        m[i] = l[i];
        m[8 + i] = r[i];
    }
    iv(out);
    compress(out, m, 0, 0, 64, PARENT | (root ? ROOT : 0));
}
__host__ static inline void hash_bytes(const uint8_t *in, size_t len, uint8_t out[32]) {
    uint32_t h[8];
    subtree(in, len, 0, true, h);
    memcpy(out, h, 32);  // little-endian host
}

}  // namespace b3
