// host_field.hpp -- host-side helpers over the f128 field: small NTTs, polynomial evaluation,
// byte conversion and the Fiat-Shamir public coin (winter-crypto DefaultRandomCoin<Blake3_256>,
// prover/src/lib.rs:45).
#pragma once
#include <stdint.h>
#include <string.h>

#include <map>
#include <utility>
#include <vector>

#include "blake3.hpp"
#include "ext2.hpp"
#include "f128.hpp"

namespace zk {

static constexpr uint64_t TWO_ADIC_ROOT_LO = 0, TWO_ADIC_ROOT_HI = 0;  // computed at startup

inline fe h_pow(fe b, uint64_t e) { return fe_exp(b, e, 0); }

// 3^((p-1)/2^40): root of unity of order 2^40 (winter-math f128 TWO_ADIC_ROOT_OF_UNITY)
inline fe h_two_adic_root() {
    // (p - 1) >> 40 = 0xffffffffffffff_ffffffffd3 ... computed from p's limbs
    const unsigned __int128 p = ((unsigned __int128)ZK_P_HI << 64) | ZK_P_LO;
    const unsigned __int128 e = (p - 1) >> 40;
    return fe_exp(fe_make(3), (uint64_t)e, (uint64_t)(e >> 64));
}

inline fe h_root_of_unity(int log_n) {
    static fe root = h_two_adic_root();
    fe r = root;
    for (int i = log_n; i < 40; i++) r = fe_mul(r, r);
    return r;
}

inline fe h_inv(fe a) { return fe_inv(a); }

// A[j] = sum_k a[k] w^(jk), natural order (iterative radix-2)
inline void h_ntt(std::vector<fe> &a, fe w) {
    size_t n = a.size();
    int lg = 0;
    while (((size_t)1 << lg) < n) lg++;
    for (size_t i = 0; i < n; i++) {
        size_t r = 0;
        for (int b = 0; b < lg; b++) r |= ((i >> b) & 1) << (lg - 1 - b);
        if (i < r) std::swap(a[i], a[r]);
    }
    for (size_t len = 2; len <= n; len <<= 1) {
        fe wl = h_pow(w, n / len);
        size_t half = len / 2;
        std::vector<fe> tw(half);
        tw[0] = fe_one();
        for (size_t j = 1; j < half; j++) tw[j] = fe_mul(tw[j - 1], wl);
        for (size_t i = 0; i < n; i += len)
            for (size_t j = 0; j < half; j++) {
                fe u = a[i + j], v = fe_mul(a[i + j + half], tw[j]);
                a[i + j] = fe_add(u, v);
                a[i + j + half] = fe_sub(u, v);
            }
    }
}

// interpolate evaluations over offset * <w_size> into coefficients (in place)
inline void h_interp_coset(std::vector<fe> &v, fe offset) {
    size_t n = v.size();
    int lg = 0;
    while (((size_t)1 << lg) < n) lg++;
    h_ntt(v, h_inv(h_root_of_unity(lg)));
    fe s = h_inv(fe_make(n)), io = h_inv(offset);
    for (size_t k = 0; k < n; k++) {
        v[k] = fe_mul(v[k], s);
        s = fe_mul(s, io);
    }
}

// h_interp_coset for offset 3 with the per-size tables (inverse twiddles per stage, n^-1 3^-k)
// cached per thread: the FRI remainder is interpolated on every proof while the GPU waits
inline void h_interp_coset3_cached(std::vector<fe> &v) {
    struct Tabs {
        std::vector<fe> tw, scale;  // tw[len/2 + j] = w_len^-j for each stage len; scale[k] = n^-1 3^-k
    };
    static thread_local std::map<size_t, Tabs> cache;
    const size_t n = v.size();
    int lg = 0;
    while (((size_t)1 << lg) < n) lg++;
    auto it = cache.find(n);
    if (it == cache.end()) {
        Tabs t;
        t.tw.assign(n, fe_zero());
        const fe wi = h_inv(h_root_of_unity(lg));
        for (size_t len = 2; len <= n; len <<= 1) {
            const fe wl = h_pow(wi, n / len);
            fe w = fe_one();
            for (size_t j = 0; j < len / 2; j++, w = fe_mul(w, wl)) t.tw[len / 2 + j] = w;
        }
        t.scale.resize(n);
        fe s = h_inv(fe_make(n));
        const fe io = h_inv(fe_make(3));
        for (size_t k = 0; k < n; k++, s = fe_mul(s, io)) t.scale[k] = s;
        it = cache.emplace(n, std::move(t)).first;
    }
    const Tabs &t = it->second;
    for (size_t i = 0; i < n; i++) {
        size_t r = 0;
        for (int b = 0; b < lg; b++) r |= ((i >> b) & 1) << (lg - 1 - b);
        if (i < r) std::swap(v[i], v[r]);
    }
    for (size_t len = 2; len <= n; len <<= 1) {
        const size_t half = len / 2;
        for (size_t i = 0; i < n; i += len)
            for (size_t j = 0; j < half; j++) {
                const fe u = v[i + j], x = fe_mul(v[i + j + half], t.tw[half + j]);
                v[i + j] = fe_add(u, x);
                v[i + j + half] = fe_sub(u, x);
            }
    }
    for (size_t k = 0; k < n; k++) v[k] = fe_mul(v[k], t.scale[k]);
}

inline fe h_poly_eval(const fe *c, size_t m, fe x) {
    fe r = fe_zero();
    for (size_t k = m; k-- > 0;) r = fe_add(fe_mul(r, x), c[k]);
    return r;
}

inline fe fe_from_bytes(const uint8_t *b) {
    fe v;
    memcpy(&v.lo, b, 8);
    memcpy(&v.hi, b + 8, 8);
    return v;
}
inline void fe_to_bytes(fe v, uint8_t *b) {
    memcpy(b, &v.lo, 8);
    memcpy(b + 8, &v.hi, 8);
}
inline bool fe_canonical(fe v) { return !(v.hi == ZK_P_HI && v.lo >= ZK_P_LO); }

inline void hash_elems(const fe *e, size_t k, uint8_t out[32]) {
    b3::hash_bytes(reinterpret_cast<const uint8_t *>(e), 16 * k, out);
}

// ---- DefaultRandomCoin<Blake3_256> ----
struct Coin {
    uint8_t seed[32];
    uint64_t counter = 0;
    void init(const std::vector<fe> &elems) {
        hash_elems(elems.data(), elems.size(), seed);
        counter = 0;
    }
    void reseed(const uint8_t d[32]) {
        uint8_t buf[64];
        memcpy(buf, seed, 32);
        memcpy(buf + 32, d, 32);
        b3::hash_bytes(buf, 64, seed);
        counter = 0;
    }
    static void merge_with_int(const uint8_t s[32], uint64_t v, uint8_t out[32]) {
        uint8_t buf[40];
        memcpy(buf, s, 32);
        memcpy(buf + 32, &v, 8);
        b3::hash_bytes(buf, 40, out);
    }
    void next(uint8_t out[32]) {
        counter++;
        merge_with_int(seed, counter, out);
    }
    fe draw() {
        for (int i = 0; i < 1000; i++) {
            uint8_t d[32];
            next(d);
            fe v = fe_from_bytes(d);
            if (fe_canonical(v)) return v;
        }
        return fe_zero();
    }
    // draw::<E>: E::ELEMENT_BYTES of the next digest, retried until every component is canonical
    // (k = 1: the first 16 bytes, identical to draw(); k = 2: both 16-byte halves)
    fe2 draw_ext(int k) {
        for (int i = 0; i < 1000; i++) {
            uint8_t d[32];
            next(d);
            const fe a = fe_from_bytes(d), b = k == 2 ? fe_from_bytes(d + 16) : fe_zero();
            if (fe_canonical(a) && fe_canonical(b)) return fe2{a, b};
        }
        return fe2_zero();
    }
};

}  // namespace zk
