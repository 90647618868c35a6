// verifier.cpp -- host verifier for the proofs this library writes: winterfell 0.9
// `verify::<ProcessorAir, Blake3_256, DefaultRandomCoin>` (call sites vm/src/lib.rs:93-98,
// examples/linear_regression/src/main.rs:85), restated for ProcessorAir and the proof layout of
// DESIGN.md "Protocol profile" (P1-P14).
//
// Both FieldExtension::None and Quadratic (every E value is an fe2; base values carry b = 0).
// Checks: proof context and conjectured security (winter-air: min(128*k - log2 N, log2(B) * q
// [+ grinding when the query bound is >= 80]) - 1), the transcript, every batch Merkle opening
// (trace, composition, FRI layers), the out-of-domain identity H(z) = sum_j z^(jn) H_j(z) against
// ProcessorAir::evaluate_transition at z (air/src/lib.rs:104-168, constrains.rs:95-216) and the
// assertions (air/src/lib.rs:170-195), the DEEP values at the query positions, every FRI fold, the
// remainder commitment and the query proof of work.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <map>
#include <string>
#include <vector>

#include "../../include/zkvm_gpu.h"
#include "air_shape.hpp"
#include "host_field.hpp"
#include "rescue_consts.hpp"

using namespace zk;

namespace {

constexpr int W = ZK_TRACE_WIDTH, NT = 20, NA = 22;

int ilog2z(size_t n) {
    int r = 0;
    while (((size_t)1 << r) < n) r++;
    return r;
}

struct Reader {
    const uint8_t *p;
    size_t len, off = 0;
    bool bad = false;
    const uint8_t *take(size_t n) {
        if (bad || off + n > len) {
            bad = true;
            return nullptr;
        }
        const uint8_t *q = p + off;
        off += n;
        return q;
    }
    uint8_t u8() {
        const uint8_t *q = take(1);
        return q ? q[0] : 0;
    }
    uint16_t u16() {
        const uint8_t *q = take(2);
        return q ? (uint16_t)(q[0] | q[1] << 8) : 0;
    }
    uint32_t u32() {
        const uint8_t *q = take(4);
        uint32_t v = 0;
        if (q) memcpy(&v, q, 4);
        return v;
    }
};

struct VerifyError {
    std::string msg;
};
[[noreturn]] void fail(const std::string &m) { throw VerifyError{m}; }

fe elem(const uint8_t *b) {
    const fe v = fe_from_bytes(b);
    if (!fe_canonical(v)) fail("non-canonical field element");
    return v;
}

void merge(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
    uint8_t buf[64];
    memcpy(buf, a, 32);
    memcpy(buf + 32, b, 32);
    b3::hash_bytes(buf, 64, out);
}

// BatchMerkleProof::get_root: the leaves at `idx` (digests in the same order) and the serialized
// per-path node vectors (MerkleTree::prove_batch order) must rebuild `root`.
void check_batch(const uint8_t *bytes, size_t blen, const std::vector<std::array<uint8_t, 32>> &leaf,
                 const std::vector<uint64_t> &idx, int depth, const uint8_t root[32], const char *what) {
    Reader r{bytes, blen};
    std::vector<uint64_t> norm;
    for (uint64_t i : idx) norm.push_back(i & ~1ULL);
    std::sort(norm.begin(), norm.end());
    norm.erase(std::unique(norm.begin(), norm.end()), norm.end());
    const size_t nv = r.u8();
    if (nv != norm.size()) fail(std::string(what) + ": wrong number of paths");
    std::vector<std::vector<std::array<uint8_t, 32>>> vec(nv);
    for (auto &v : vec) {
        const size_t k = r.u8();
        for (size_t t = 0; t < k; t++) {
            const uint8_t *d = r.take(32);
            if (!d) fail(std::string(what) + ": truncated path");
            std::array<uint8_t, 32> a;
            memcpy(a.data(), d, 32);
            v.push_back(a);
        }
    }
    if (r.bad || r.off != r.len) fail(std::string(what) + ": malformed batch proof");
    auto leaf_of = [&](uint64_t i) -> const uint8_t * {
        for (size_t t = 0; t < idx.size(); t++)
            if (idx[t] == i) return leaf[t].data();
        return nullptr;
    };
    const uint64_t nleaves = 1ULL << depth;
    std::map<uint64_t, std::array<uint8_t, 32>> nodes;
    std::vector<size_t> used(nv, 0);
    std::vector<uint64_t> next;
    for (size_t i = 0; i < nv; i++) {
        const uint8_t *l0 = leaf_of(norm[i]), *l1 = leaf_of(norm[i] + 1);
        if (!l0) {
            if (used[i] >= vec[i].size()) fail(std::string(what) + ": missing sibling");
            l0 = vec[i][used[i]++].data();
        }
        if (!l1) {
            if (used[i] >= vec[i].size()) fail(std::string(what) + ": missing sibling");
            l1 = vec[i][used[i]++].data();
        }
        std::array<uint8_t, 32> par;
        merge(l0, l1, par.data());
        const uint64_t k = (nleaves + norm[i]) >> 1;
        nodes[k] = par;
        next.push_back(k);
    }
    for (int lvl = 1; lvl < depth; lvl++) {
        std::vector<uint64_t> cur = next;
        next.clear();
        for (size_t i = 0; i < cur.size(); i++) {
            const uint64_t node = cur[i], sib = node ^ 1;
            const uint8_t *sd;
            if (i + 1 < cur.size() && cur[i + 1] == sib) {
                sd = nodes[sib].data();
                i++;
            } else {
                if (used[i] >= vec[i].size()) fail(std::string(what) + ": path too short");
                sd = vec[i][used[i]++].data();
            }
            std::array<uint8_t, 32> par;
            if (node & 1) merge(sd, nodes[node].data(), par.data());
            else merge(nodes[node].data(), sd, par.data());
            nodes[node >> 1] = par;
            next.push_back(node >> 1);
        }
    }
    auto it = nodes.find(1);
    if (it == nodes.end() || memcmp(it->second.data(), root, 32)) fail(std::string(what) + " does not match the commitment");
}

fe mds_entry(const uint64_t m[16][2], int i) { return fe_make(m[i][0], m[i][1]); }
fe2 cube(fe2 x) { return fe2_mul(fe2_mul(x, x), x); }

// ProcessorAir::evaluate_transition (air/src/lib.rs:104-168) at one frame over E (the verifier's
// evaluate_transition<E>, E = f128 or its quadratic extension); per = 9 periodic values
void air_eval(const fe2 *cur, const fe2 *nxt, const fe2 *per, uint32_t L, fe delta, fe2 *out) {
    const fe2 one = fe2_one();
    auto nt = [&](fe2 b) { return fe2_sub(one, b); };
    auto mul = fe2_mul;
    auto add = fe2_add;
    auto sub = fe2_sub;
    const fe2 b0 = cur[5], b1 = cur[4], b2 = cur[3], b3 = cur[2], b4 = cur[1];
    auto sel = [&](fe2 a, fe2 b, fe2 c, fe2 d, fe2 e) { return mul(mul(mul(mul(a, b), c), d), e); };
    const fe2 is_add = sel(nt(b0), b1, nt(b2), nt(b3), nt(b4)), is_sadd = sel(nt(b0), b1, nt(b2), b3, nt(b4));
    const fe2 is_add2 = sel(nt(b0), b1, nt(b2), b3, b4), is_mul = sel(nt(b0), b1, nt(b2), nt(b3), b4);
    const fe2 is_smul = sel(nt(b0), b1, b2, nt(b3), nt(b4)), is_push = sel(b0, nt(b1), nt(b2), nt(b3), nt(b4));
    const fe2 is_read = sel(b0, nt(b1), nt(b2), nt(b3), b4), is_read2 = sel(b0, nt(b1), nt(b2), b3, nt(b4));
    const fe2 is_noop = sel(nt(b0), nt(b1), nt(b2), nt(b3), nt(b4));
    fe2 opcode = b0;
    for (fe2 b : {b1, b2, b3, b4}) opcode = add(add(opcode, opcode), b);
    const fe2 *s = cur + 12, *sn = nxt + 12;
    const fe four = fe_make(4);
    out[0] = sub(nxt[0], add(cur[0], one));
    out[1] = add(sub(add(sub(sub(nxt[11], cur[11]), b0), b1), fe2_mulb(is_read2, four)), fe2_mulb(is_add2, four));
    out[2] = mul(b0, b1);
    out[3] = mul(is_add, sub(sn[0], add(s[0], s[1])));
    fe2 a4 = fe2_zero(), a5 = fe2_zero(), a7 = fe2_zero();
    for (uint32_t i = 0; i < L; i++) {
        const fe2 triv = i == L - 1 ? fe2_mulb(s[0], delta) : fe2_zero();  // encrypt_trivial (server_key.rs)
        a4 = add(a4, sub(sn[i], add(s[1 + i], triv)));
        a5 = add(a5, sub(sn[i], add(s[i], s[L + i])));
        a7 = add(a7, sub(sn[i], mul(s[1 + i], s[0])));
    }
    out[4] = mul(is_sadd, a4);
    out[5] = mul(is_add2, a5);
    out[6] = mul(is_mul, sub(sn[0], mul(s[0], s[1])));
    out[7] = mul(is_smul, a7);
    out[8] = mul(is_push, sub(sn[1], s[0]));
    out[9] = mul(is_read, sub(sn[1], s[0]));
    out[10] = mul(is_read2, sub(sn[5], s[0]));
    out[11] = mul(is_noop, sub(sn[0], s[0]));
    const fe2 hf = per[0], h0 = cur[6];
    fe2 x[4], m0[4], y[4];
    for (int i = 0; i < 4; i++) x[i] = cube(cur[7 + i]);
    for (int i = 0; i < 4; i++) {
        fe2 t = fe2_zero();
        for (int j = 0; j < 4; j++) t = add(t, fe2_mulb(x[j], mds_entry(ZK_MDS, 4 * i + j)));
        m0[i] = add(t, per[1 + i]);
    }
    m0[0] = add(m0[0], opcode);
    m0[1] = add(m0[1], mul(sn[0], is_push));
    for (int i = 0; i < 4; i++) y[i] = sub(nxt[7 + i], per[5 + i]);
    for (int i = 0; i < 4; i++) {
        fe2 t = fe2_zero();
        for (int j = 0; j < 4; j++) t = add(t, fe2_mulb(y[j], mds_entry(ZK_INV_MDS, 4 * i + j)));
        out[12 + i] = mul(mul(sub(cube(t), m0[i]), hf), h0);
    }
    const fe2 nf = sub(one, hf);
    out[16] = mul(mul(sub(nxt[7], cur[7]), nf), h0);
    out[17] = mul(mul(sub(nxt[8], cur[8]), nf), h0);
    out[18] = mul(mul(nxt[9], nf), h0);
    out[19] = mul(mul(nxt[10], nf), h0);
}

// periodic columns (CYCLE_MASK + 8 ARK columns, air/src/lib.rs:201-225) at a point y = z^(n/16)
void periodic_at(fe2 y, fe2 out[9]) {
    std::vector<std::vector<fe>> cols(9, std::vector<fe>(16));
    for (int r = 0; r < 16; r++) {
        cols[0][r] = fe_make(r < 14 ? 1 : 0);
        for (int c = 0; c < 8; c++) cols[1 + c][r] = fe_make(ZK_ARK[8 * r + c][0], ZK_ARK[8 * r + c][1]);
    }
    for (int j = 0; j < 9; j++) {
        h_interp_coset(cols[j], fe_one());
        fe2 acc = fe2_zero();
        for (int t = 16; t-- > 0;) acc = fe2_add(fe2_mul(acc, y), fe2_lift(cols[j][t]));
        out[j] = acc;
    }
}

// k base components per E value (the wire order), canonical or the proof is rejected
fe2 elem_ext(const uint8_t *b, int k) { return fe2{elem(b), k == 2 ? elem(b + 16) : fe_zero()}; }
void flatten(const fe2 *v, size_t m, int k, std::vector<fe> &out) {
    out.clear();
    for (size_t i = 0; i < m; i++) {
        out.push_back(v[i].a);
        if (k == 2) out.push_back(v[i].b);
    }
}
void hash_ext(const fe2 *v, size_t m, int k, uint8_t d[32]) {
    std::vector<fe> f;
    flatten(v, m, k, f);
    hash_elems(f.data(), f.size(), d);
}
// sum_t c[t] x^t for E coefficients at a base point
fe2 poly_eval_ext(const fe2 *c, size_t m, fe x) {
    fe2 acc = fe2_zero();
    for (size_t t = m; t-- > 0;) acc = fe2_add(fe2_mulb(acc, x), c[t]);
    return acc;
}

void verify(const uint8_t *proof, size_t plen, const zk_pub_inputs *pub, uint32_t min_security) {
    Reader r{proof, plen};
    const uint8_t width = r.u8(), auxw = r.u8(), auxr = r.u8(), logn = r.u8();
    r.take(r.u16());
    const uint8_t mlen = r.u8();
    const uint8_t *mod = r.take(mlen);
    const uint8_t nq = r.u8(), B = r.u8(), grind = r.u8(), ext = r.u8(), fold = r.u8(), remdeg = r.u8();
    const uint8_t nu = r.u8();
    if (r.bad || width != W || auxw || auxr || mlen != 16 || (ext != 1 && ext != 2) || logn < 4 || logn > 32 ||
        B < 8 || (B & (B - 1)) || !(fold == 2 || fold == 4 || fold == 8 || fold == 16) || ((remdeg + 1) & remdeg))
        fail("malformed proof context");
    uint64_t pm[2] = {ZK_P_LO, ZK_P_HI};
    if (memcmp(mod, pm, 16)) fail("field modulus mismatch");
    const int K = ext;  // FieldExtension degree: 1 = None, 2 = Quadratic
    const size_t n = (size_t)1 << logn, N = n * B;
    const int logB = ilog2z(B), logN = logn + logB;
    {
        int q_sec = logB * nq;
        if (q_sec >= 80) q_sec += grind;
        const int sec = std::min(std::min(128 * K - logN, q_sec) - 1, 128);
        if (sec < (int)min_security) fail("insufficient proof security: " + std::to_string(sec));
    }
    int nl = 0;
    for (size_t s = N; s > (size_t)(remdeg + 1) * B; s /= fold) nl++;
    const uint16_t clen = r.u16();
    const uint8_t *coms = r.take(clen);
    if (r.bad || clen != 32 * (2 + nl + 1)) fail("malformed commitments");

    // transcript [P1-P8]
    Coin coin;
    {
        std::vector<fe> e = {fe_make((uint64_t)W << 16), fe_make(n), fe_make(ZK_P_LO), fe_make(ZK_P_HI),
                             fe_make(((uint64_t)ext << 16) | ((uint64_t)fold << 8) | remdeg), fe_make(grind),
                             fe_make(B), fe_make(nq)};
        for (int i = 0; i < 2; i++) e.push_back(fe_from_bytes(pub->program_hash[i]));
        for (int i = 0; i < 16; i++) e.push_back(fe_from_bytes(pub->stack_outputs[i]));
        coin.init(e);
    }
    coin.reseed(coms);
    fe2 ct[NT], cb[NA];
    for (auto &v : ct) v = coin.draw_ext(K);
    for (auto &v : cb) v = coin.draw_ext(K);
    coin.reseed(coms + 32);
    const fe2 z = coin.draw_ext(K);

    if (r.u8() != 1) fail("expected one trace segment");
    const uint32_t tvl = r.u32();
    const uint8_t *tv = r.take(tvl);
    const uint32_t tpl = r.u32();
    const uint8_t *tp = r.take(tpl);
    const uint32_t cvl = r.u32();
    const uint8_t *cv = r.take(cvl);
    const uint32_t cpl = r.u32();
    const uint8_t *cp = r.take(cpl);
    const uint16_t tsl = r.u16();
    const uint8_t *ts = r.take(tsl);
    const uint16_t oel = r.u16();
    const uint8_t *oe = r.take(oel);
    const int ES = 16 * K;  // bytes per E value
    if (r.bad || tsl != 1 + 2 * W * ES || ts[0] != 2 || oel == 0 || oel % ES || oel / ES > ZK_MAX_CCOLS)
        fail("malformed out-of-domain frame");
    const int C = oel / ES;
    // the composition column count follows from the AIR (winter-air derives it from the context)
    if (C != zk::num_comp_cols(n)) fail("malformed out-of-domain frame");
    std::vector<fe2> ood(2 * W + C);
    for (int c = 0; c < W; c++) {
        ood[c] = elem_ext(ts + 1 + 2 * ES * c, K);
        ood[W + c] = elem_ext(ts + 1 + 2 * ES * c + ES, K);
    }
    for (int j = 0; j < C; j++) ood[2 * W + j] = elem_ext(oe + ES * j, K);
    {
        uint8_t d[32];
        hash_ext(ood.data(), 2 * W, K, d);
        coin.reseed(d);
        hash_ext(ood.data() + 2 * W, C, K, d);
        coin.reseed(d);
    }
    // out-of-domain identity
    if (!zk::ood_identity(ood.data(), C, ct, cb, z, n, pub)) fail("out-of-domain constraint evaluation mismatch");
    fe2 at[W], ac[ZK_MAX_CCOLS];
    for (auto &v : at) v = coin.draw_ext(K);
    for (int j = 0; j < C; j++) ac[j] = coin.draw_ext(K);
    std::vector<fe2> alphas(nl);
    for (int l = 0; l < nl; l++) {
        coin.reseed(coms + 64 + 32 * l);
        alphas[l] = coin.draw_ext(K);
    }
    coin.reseed(coms + 64 + 32 * nl);

    if (r.u8() != nl) fail("wrong number of FRI layers");
    std::vector<const uint8_t *> lv(nl), lp(nl);
    std::vector<uint32_t> lvl(nl), lpl(nl);
    for (int l = 0; l < nl; l++) {
        lvl[l] = r.u32();
        lv[l] = r.take(lvl[l]);
        lpl[l] = r.u32();
        lp[l] = r.take(lpl[l]);
    }
    const uint16_t rml = r.u16();
    const uint8_t *rm = r.take(rml);
    const uint8_t nparts = r.u8();
    const uint8_t *nonce_b = r.take(8);
    const uint8_t gkr = r.u8();
    if (r.bad || nparts != 0 || gkr != 0 || r.off != r.len || rml % ES) fail("malformed proof tail");
    {
        uint8_t d[32];
        b3::hash_bytes(rm, rml, d);
        if (memcmp(d, coms + 64 + 32 * nl, 32)) fail("remainder commitment mismatch");
    }
    // proof of work and query positions [P10, P11]
    uint64_t nonce;
    memcpy(&nonce, nonce_b, 8);
    {
        uint8_t d[32];
        Coin::merge_with_int(coin.seed, nonce, d);
        uint64_t head;
        memcpy(&head, d, 8);
        if ((head ? (unsigned)__builtin_ctzll(head) : 64u) < grind) fail("query seed proof of work is invalid");
        memcpy(coin.seed, d, 32);
        coin.counter = 0;
    }
    std::vector<uint64_t> pos;
    for (int q = 0; q < nq; q++) {
        uint8_t d[32];
        coin.next(d);
        uint64_t v;
        memcpy(&v, d, 8);
        pos.push_back(v & (N - 1));
    }
    std::sort(pos.begin(), pos.end());
    pos.erase(std::unique(pos.begin(), pos.end()), pos.end());
    if (pos.size() != nu) fail("number of unique queries mismatch");
    const int CK = C * K;
    if (tvl != nu * W * 16u || cvl != nu * (uint32_t)CK * 16u) fail("malformed query values");
    std::vector<fe> tvals(nu * W), cflat(nu * CK);
    for (size_t i = 0; i < tvals.size(); i++) tvals[i] = elem(tv + 16 * i);
    for (size_t i = 0; i < cflat.size(); i++) cflat[i] = elem(cv + 16 * i);
    std::vector<std::array<uint8_t, 32>> dig(nu);
    for (size_t q = 0; q < nu; q++) hash_elems(tvals.data() + q * W, W, dig[q].data());
    check_batch(tp, tpl, dig, pos, logN, coms, "trace query");
    for (size_t q = 0; q < nu; q++) hash_elems(cflat.data() + q * CK, CK, dig[q].data());
    check_batch(cp, cpl, dig, pos, logN, coms + 32, "constraint query");

    // DEEP values at the positions (in E)
    std::vector<fe2> evals(nu);
    {
        const fe wN = h_root_of_unity(logN), three = fe_make(3);
        const fe2 zg = fe2_mulb(z, h_root_of_unity(logn));
        for (size_t q = 0; q < nu; q++) {
            const fe2 x = fe2_lift(fe_mul(three, h_pow(wN, pos[q])));
            fe2 s1 = fe2_zero(), s2 = fe2_zero();
            for (int c = 0; c < W; c++) {
                const fe2 v = fe2_lift(tvals[q * W + c]);
                s1 = fe2_add(s1, fe2_mul(at[c], fe2_sub(v, ood[c])));
                s2 = fe2_add(s2, fe2_mul(at[c], fe2_sub(v, ood[W + c])));
            }
            for (int j = 0; j < C; j++) {
                const fe *hv = cflat.data() + q * CK + j * K;
                const fe2 h = fe2{hv[0], K == 2 ? hv[1] : fe_zero()};
                s1 = fe2_add(s1, fe2_mul(ac[j], fe2_sub(h, ood[2 * W + j])));
            }
            evals[q] = fe2_add(fe2_mul(s1, fe2_inv(fe2_sub(x, z))), fe2_mul(s2, fe2_inv(fe2_sub(x, zg))));
        }
    }
    // FRI [P9]
    size_t dsz = N;
    std::vector<uint64_t> fp = pos;
    fe dgen = h_root_of_unity(logN);
    for (int l = 0; l < nl; l++) {
        const size_t target = dsz / fold;
        std::vector<uint64_t> folded;
        for (uint64_t p : fp)
            if (std::find(folded.begin(), folded.end(), p % target) == folded.end()) folded.push_back(p % target);
        const size_t m = folded.size();
        if (lvl[l] != m * fold * ES) fail("malformed FRI layer " + std::to_string(l));
        std::vector<fe2> rows(m * fold);
        for (size_t i = 0; i < rows.size(); i++) rows[i] = elem_ext(lv[l] + ES * i, K);
        std::vector<std::array<uint8_t, 32>> ld(m);
        for (size_t q = 0; q < m; q++) hash_ext(rows.data() + q * fold, fold, K, ld[q].data());
        check_batch(lp[l], lpl[l], ld, folded, ilog2z(target), coms + 64 + 32 * l,
                    ("FRI layer " + std::to_string(l) + " query").c_str());
        for (size_t i = 0; i < fp.size(); i++) {
            const size_t ri = std::find(folded.begin(), folded.end(), fp[i] % target) - folded.begin();
            if (!fe2_eq(rows[ri * fold + fp[i] / target], evals[i])) fail("FRI layer " + std::to_string(l) + " folding mismatch");
        }
        std::vector<fe2> nxt(m);
        for (size_t q = 0; q < m; q++) {
            // interpolate each E component over the coset, then evaluate the E polynomial at alpha
            std::vector<fe> va(fold), vb(fold);
            for (int t = 0; t < fold; t++) {
                va[t] = rows[q * fold + t].a;
                vb[t] = rows[q * fold + t].b;
            }
            const fe xo = fe_mul(fe_make(3), h_pow(dgen, folded[q]));
            h_interp_coset(va, xo);
            if (K == 2) h_interp_coset(vb, xo);
            fe2 acc = fe2_zero();
            for (int t = fold; t-- > 0;) acc = fe2_add(fe2_mul(acc, alphas[l]), fe2{va[t], K == 2 ? vb[t] : fe_zero()});
            nxt[q] = acc;
        }
        evals = nxt;
        fp = folded;
        dgen = h_pow(dgen, fold);
        dsz = target;
    }
    const size_t rem_len = rml / ES;
    if (rem_len != dsz / B) fail("remainder has the wrong size");
    std::vector<fe2> rem(rem_len);
    for (size_t i = 0; i < rem_len; i++) rem[i] = elem_ext(rm + ES * i, K);
    for (size_t i = 0; i < fp.size(); i++) {
        const fe x = fe_mul(fe_make(3), h_pow(dgen, fp[i]));
        if (!fe2_eq(poly_eval_ext(rem.data(), rem_len, x), evals[i])) fail("FRI remainder mismatch");
    }
}

}  // namespace


// The verifier's out-of-domain identity (winterfell verifier: evaluate_constraints at z against the
// composition columns): sum_k ct_k C_k(z) * divisor(z) + boundary terms == sum_j z^(jn) H_j(z).
// ood = [T(z)]_W ++ [T(zg)]_W ++ [H_j(z)]_C.  The prover runs it as its degree check.
bool zk::ood_identity(const fe2 *ood, int C, const fe2 *ct, const fe2 *cb, fe2 z, size_t n, const zk_pub_inputs *pub) {
    const int logn = ilog2z(n);
    const fe g = h_root_of_unity(logn);
    const fe2 one = fe2_one();
    fe2 per[9], ev[NT];
    periodic_at(fe2_exp(z, n / 16), per);
    air_eval(ood, ood + W, per, pub->lwe_size, fe_make(pub->delta), ev);
    fe2 t = fe2_zero();
    for (int k = 0; k < NT; k++) t = fe2_add(t, fe2_mul(ct[k], ev[k]));
    const fe2 gl2 = fe2_lift(h_pow(g, n - 2)), gl1 = fe2_lift(h_pow(g, n - 1)), zn = fe2_exp(z, n);
    fe2 h = fe2_mul(fe2_mul(t, fe2_mul(fe2_sub(z, gl2), fe2_sub(z, gl1))), fe2_inv(fe2_sub(zn, one)));
    const int fc[12] = {0, 7, 8, 11, 12, 13, 14, 15, 16, 17, 18, 19};
    fe2 bs0 = fe2_zero(), bs1 = fe2_zero();
    for (int i = 0; i < 12; i++) bs0 = fe2_add(bs0, fe2_mul(cb[i], ood[fc[i]]));
    for (int i = 0; i < 2; i++)
        bs1 = fe2_add(bs1, fe2_mul(cb[12 + i], fe2_sub(ood[7 + i], fe2_lift(fe_from_bytes(pub->program_hash[i])))));
    for (int i = 0; i < 8; i++)
        bs1 = fe2_add(bs1, fe2_mul(cb[14 + i], fe2_sub(ood[12 + i], fe2_lift(fe_from_bytes(pub->stack_outputs[i])))));
    h = fe2_add(h, fe2_mul(bs0, fe2_inv(fe2_sub(z, one))));
    h = fe2_add(h, fe2_mul(bs1, fe2_inv(fe2_sub(z, gl2))));
    fe2 hc = fe2_zero(), zz = one;
    for (int j = 0; j < C; j++) {
        hc = fe2_add(hc, fe2_mul(zz, ood[2 * W + j]));
        zz = fe2_mul(zz, zn);
    }
    return fe2_eq(h, hc);
}

int zk_verify(const uint8_t *proof, size_t proof_len, const zk_pub_inputs *pub, uint32_t min_security, char *msg,
              size_t msg_cap) {
    if (msg && msg_cap) msg[0] = 0;
    if (!proof || !pub) {
        if (msg && msg_cap) snprintf(msg, msg_cap, "null argument");
        return ZK_ERR_INVALID_ARG;
    }
    // air_eval indexes the OOD frame by lwe_size: the same bound (and message) as the prover
    if (pub->lwe_size == 0 || pub->lwe_size > 5) {
        if (msg && msg_cap)
            snprintf(msg, msg_cap, "lwe_size must be in [1, 5] (enforce_add2 reads 2*lwe_size stack items, constrains.rs:129)");
        return ZK_ERR_INVALID_ARG;
    }
    try {
        verify(proof, proof_len, pub, min_security);
    } catch (const VerifyError &e) {
        if (msg && msg_cap) snprintf(msg, msg_cap, "%s", e.msg.c_str());
        return ZK_ERR_VERIFY;
    }
    return ZK_OK;
}
