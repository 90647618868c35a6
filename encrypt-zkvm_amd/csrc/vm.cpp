// vm.cpp -- host-side VM front end and trace generator (harness of the prove path).
//
// The reference produces the 28-column trace on the CPU before calling Prover::prove
// (vm/src/lib.rs:13-18); this file is that caller, restated in C++ with the same four state
// machines so that benchmarks and tests can build real, AIR-satisfying traces of any size:
//   Program::compile ....... vm/src/program/mod.rs:37-131 (padding: PUSH aligned to 8, no op in
//                            cycle slots 14/15, final pad to a multiple of 16; Rescue program hash)
//   Processor::run/trace ... vm/src/processor/mod.rs:61-95
//   System / Decoder / Chiplets / Stack ... vm/src/processor/{system,decoder,chiplets,stack}.rs
// Error texts match the reference's Display impls (vm/src/program/errors.rs, processor/errors.rs).
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/zkvm_gpu.h"
#include "host_field.hpp"
#include "rescue_consts.hpp"

using namespace zk;

namespace {

thread_local std::string vm_err;

enum : uint8_t { NOOP = 0x00, PUSH = 0x10, READ = 0x11, READ2 = 0x12, ADD = 0x08, MUL = 0x09, SADD = 0x0a,
                 SMUL = 0x0c, ADD2 = 0x0b };
constexpr int CYCLE = 16, NUM_ROUNDS = 14, MAX_STACK = 16, MIN_TRACE = 16;

struct Op {
    uint8_t code, value;
};

std::string op_str(Op o) {
    switch (o.code) {
    case NOOP: return "noop";
    case PUSH: return "push(" + std::to_string(o.value) + ")";
    case READ: return "read";
    case READ2: return "read2";
    case ADD: return "add";
    case MUL: return "mul";
    case SADD: return "sadd";
    case SMUL: return "smul";
    case ADD2: return "add2";
    }
    return "?";
}

fe mds(const uint64_t m[16][2], int i) { return fe_make(m[i][0], m[i][1]); }

// The S-box chains of the four state elements are independent: each step below runs the four
// lanes back to back (lane loop innermost), which lets the out-of-order core overlap the four
// multiply chains (~4.4 ns per product instead of ~10 for one chain).
__attribute__((noinline)) void sqn4(fe v[4], int k) {  // v^(2^k)
    for (int t = 0; t < k; t++)
        for (int i = 0; i < 4; i++) v[i] = fe_mul(v[i], v[i]);
}
__attribute__((noinline)) void mul4(fe v[4], const fe w[4]) {
    for (int i = 0; i < 4; i++) v[i] = fe_mul(v[i], w[i]);
}
inline void cp4(fe d[4], const fe s[4]) {
    for (int i = 0; i < 4; i++) d[i] = s[i];
}
// x^(1/3) = x^INV_ALPHA for 4 elements (crypto/src/rescue.rs:154-160, INV_ALPHA = (2p - 1)/3
// = 0xaaaaaaaaaaaaaaaa_aaaa8caaaaaaaaab) by an addition chain over the repeated "10" bit pairs:
// w_k = x^("10" x k), w_2k = w_k^(4^k) w_k; 136 squarings + 13 multiplies instead of ~190 products.
inline void cube_root4(fe s[4]) {
    fe x[4], w1[4], w2[4], w4[4], w8[4], w16[4], r[4], t[4], u[4];
    cp4(x, s);
    cp4(w1, x);
    sqn4(w1, 1);  // "10"
    cp4(w2, w1);
    sqn4(w2, 2);
    mul4(w2, w1);  // 0xa
    cp4(w4, w2);
    sqn4(w4, 4);
    mul4(w4, w2);  // 0xaa
    cp4(w8, w4);
    sqn4(w8, 8);
    mul4(w8, w4);  // 0xaaaa
    cp4(w16, w8);
    sqn4(w16, 16);
    mul4(w16, w8);  // 0xaaaaaaaa
    cp4(r, w16);
    sqn4(r, 32);
    mul4(r, w16);  // 0xaaaaaaaaaaaaaaaa
    sqn4(r, 16);
    mul4(r, w8);  // 20 hex digits 'a'
    cp4(u, w1);  // x^0x8c = ((x^2)^16 * x^3)^4
    mul4(u, x);
    cp4(t, w1);
    sqn4(t, 4);
    mul4(t, u);
    sqn4(t, 2);
    sqn4(r, 8);
    mul4(r, t);  // ... 8c
    cp4(t, w16);  // 9 hex digits 'a' = 0xaaaaaaaa << 4 | 0xa
    sqn4(t, 4);
    mul4(t, w2);
    sqn4(r, 36);
    mul4(r, t);
    cp4(t, w2);  // 0xb = 0xa + 1
    mul4(t, x);
    sqn4(r, 4);
    mul4(r, t);
    cp4(s, r);
}

// Rescue128 (crypto/src/rescue.rs:30-56, 102-118)
struct Rescue {
    fe s[4] = {fe_zero(), fe_zero(), fe_zero(), fe_zero()};
    uint64_t step = 0;
    static void mds_mul(fe *v) {
        fe r[4];
        for (int i = 0; i < 4; i++) {
            r[i] = fe_zero();
            for (int j = 0; j < 4; j++) r[i] = fe_add(r[i], fe_mul(mds(ZK_MDS, 4 * i + j), v[j]));
        }
        memcpy(v, r, sizeof r);
    }
    void round(uint8_t code, uint8_t value) {
        int r = (int)(step % CYCLE);
        for (auto &x : s) x = fe_mul(fe_mul(x, x), x);
        mds_mul(s);
        for (int i = 0; i < 4; i++) s[i] = fe_add(s[i], fe_make(ZK_ARK[8 * r + i][0], ZK_ARK[8 * r + i][1]));
        s[0] = fe_add(s[0], fe_make(code));
        s[1] = fe_add(s[1], fe_make(value));
        cube_root4(s);  // x^(1/3): INV_ALPHA = 226854911280625642308916371969163307691
        mds_mul(s);
        for (int i = 0; i < 4; i++) s[i] = fe_add(s[i], fe_make(ZK_ARK[8 * r + 4 + i][0], ZK_ARK[8 * r + 4 + i][1]));
    }
    bool is_round() const { return step % CYCLE < NUM_ROUNDS; }
    void update(uint8_t code, uint8_t value) {
        if (is_round())
            round(code, value);
        else
            s[2] = s[3] = fe_zero();
        step++;
    }
};

std::string trim(const std::string &x) {
    size_t a = x.find_first_not_of(" \t\r\n\v\f"), b = x.find_last_not_of(" \t\r\n\v\f");
    return a == std::string::npos ? "" : x.substr(a, b - a + 1);
}

// Tokenize, parse and pad.  The program hash (Rescue over the padded code, mod.rs:88-95) is not computed
// here: the processor's chiplet absorbs the same ops in the same order, so its final sponge state is it.
int compile(const std::string &src, std::vector<Op> &code) {
    std::vector<std::string> toks;
    size_t start = 0;
    while (start <= src.size()) {
        size_t nl = src.find('\n', start);
        std::string line = trim(src.substr(start, nl == std::string::npos ? std::string::npos : nl - start));
        if (!line.empty() && line[0] != '#') {
            size_t h = line.find('#');
            if (h != std::string::npos) line = trim(line.substr(0, h));
            if (!line.empty()) toks.push_back(line);
        }
        if (nl == std::string::npos) break;
        start = nl + 1;
    }
    if (toks.empty()) {
        vm_err = "program error at 0: a program must contain at least one instruction";
        return ZK_ERR_PROGRAM;
    }
    auto pad16 = [](size_t len) { return len + (CYCLE - len % CYCLE); };
    for (size_t i = 0; i < toks.size(); i++) {
        const size_t step = i + 1;
        std::vector<std::string> parts;
        size_t a = 0;
        for (;;) {
            size_t d = toks[i].find('.', a);
            parts.push_back(toks[i].substr(a, d == std::string::npos ? std::string::npos : d - a));
            if (d == std::string::npos) break;
            a = d + 1;
        }
        static const std::pair<const char *, uint8_t> tab[] = {{"push", PUSH}, {"read", READ}, {"read2", READ2},
                                                               {"add", ADD},   {"mul", MUL},   {"sadd", SADD},
                                                               {"smul", SMUL}, {"add2", ADD2}};
        int found = -1;
        for (int t = 0; t < 8; t++)
            if (parts[0] == tab[t].first) found = t;
        if (found < 0) {
            vm_err = "program error at " + std::to_string(step) + ": instruction " + toks[i] + " is invalid";
            return ZK_ERR_PROGRAM;
        }
        Op op{tab[found].second, 0};
        if (op.code == PUSH) {
            if (parts.size() == 1) {
                vm_err = "program error at " + std::to_string(step) + ": malformed instruction push, parameter is missing";
                return ZK_ERR_PROGRAM;
            }
            if (parts.size() > 2) {
                vm_err = "program error at " + std::to_string(step) +
                         ": malformed instruction push, too many parameters provided";
                return ZK_ERR_PROGRAM;
            }
            const std::string &d = parts[1];
            size_t k = (!d.empty() && d[0] == '+') ? 1 : 0;
            bool ok = k < d.size();
            unsigned v = 0;
            for (; k < d.size() && ok; k++) {
                if (d[k] < '0' || d[k] > '9') ok = false;
                else if ((v = v * 10 + (unsigned)(d[k] - '0')) > 255) ok = false;
            }
            if (!ok) {
                vm_err = "program error at " + std::to_string(step) + ": malformed instruction push, parameter '" + d +
                         "' is invalid";
                return ZK_ERR_PROGRAM;
            }
            op.value = (uint8_t)v;
            code.resize(code.size() + (8 - code.size() % 8) % 8, Op{NOOP, 0});
        } else if (parts.size() > 1) {
            vm_err = "program error at " + std::to_string(step) + ": malformed instruction " + parts[0] +
                     ", too many parameters provided";
            return ZK_ERR_PROGRAM;
        }
        if (code.size() % CYCLE >= NUM_ROUNDS) code.resize(pad16(code.size()), Op{NOOP, 0});
        code.push_back(op);
    }
    code.resize(pad16(code.size()), Op{NOOP, 0});
    return ZK_OK;
}

// Processor::run -> trace.  Column-major output (28 x n).
struct Processor {
    size_t cap = MIN_TRACE;
    size_t clk = 0, depth = 0;
    std::vector<std::vector<fe>> reg = std::vector<std::vector<fe>>(MAX_STACK, std::vector<fe>(MIN_TRACE, fe_zero()));
    std::vector<fe> helper = std::vector<fe>(MIN_TRACE, fe_zero());
    std::vector<std::vector<fe>> bits = std::vector<std::vector<fe>>(5, std::vector<fe>(MIN_TRACE, fe_zero()));
    std::vector<fe> hflag = std::vector<fe>(MIN_TRACE, fe_zero());
    std::vector<std::vector<fe>> sponge = std::vector<std::vector<fe>>(4, std::vector<fe>(MIN_TRACE, fe_zero()));
    Rescue rescue;

    void grow() {
        if (clk < cap) return;
        cap *= 2;
        for (auto &c : reg) c.resize(cap, fe_zero());
        helper.resize(cap, fe_zero());
        for (auto &c : bits) c.resize(cap, fe_zero());
        hflag.resize(cap, fe_zero());
        for (auto &c : sponge) c.resize(cap, fe_zero());
    }

    int run(const std::vector<Op> &code, const uint8_t *pub, size_t npub, const fe *sec, size_t nsec, uint32_t L,
            uint32_t delta) {
        size_t ta = 0, tb = 0;
        for (const Op &o : code) {
            clk++;
            grow();
            auto R = [&](size_t i, size_t c) -> fe & { return reg[i][c]; };
            auto stack_err = [&](const char *what) {
                vm_err = "stack error at " + std::to_string(clk) + ": " + what;
                return ZK_ERR_STACK;
            };
            switch (o.code) {
            case NOOP:
                for (size_t i = 0; i < depth; i++) R(i, clk) = R(i, clk - 1);
                break;
            case PUSH:
            case READ:
            case READ2: {
                size_t cnt = o.code == READ2 ? L : 1;
                if (o.code == READ2 && tb >= nsec) return stack_err(("no more inputs to " + op_str(o)).c_str());
                depth += cnt;
                if (depth > (size_t)MAX_STACK) return stack_err((op_str(o) + " operation stack overflow").c_str());
                if (o.code == READ && ta >= npub) return stack_err(("no more inputs to " + op_str(o)).c_str());
                for (size_t i = 0; i < depth - cnt; i++) R(i + cnt, clk) = R(i, clk - 1);
                if (o.code == PUSH) R(0, clk) = fe_make(o.value);
                else if (o.code == READ) R(0, clk) = fe_make(pub[ta++]);
                else {
                    for (size_t i = 0; i < L; i++) R(i, clk) = sec[tb * L + i];
                    tb++;
                }
                break;
            }
            default: {
                size_t need = (o.code == ADD || o.code == MUL) ? 2 : o.code == ADD2 ? 2 * L : L + 1;
                size_t pos = o.code == ADD2 ? L : 1;
                if (depth < need) return stack_err((op_str(o) + " operation stack underflow").c_str());
                fe s0 = R(0, clk - 1);
                if (o.code == ADD) R(0, clk) = fe_add(s0, R(1, clk - 1));
                else if (o.code == MUL) R(0, clk) = fe_mul(s0, R(1, clk - 1));
                else if (o.code == SADD) {  // ServerKey::scalar_add (fhe/src/server_key.rs:104-114)
                    for (size_t i = 0; i < L; i++) {
                        fe v = R(1 + i, clk - 1);
                        if (i == L - 1) v = fe_add(v, fe_mul(fe_make(delta), s0));
                        R(i, clk) = v;
                    }
                } else if (o.code == SMUL) {  // ServerKey::scalar_mul (server_key.rs:116-124)
                    for (size_t i = 0; i < L; i++) R(i, clk) = fe_mul(R(1 + i, clk - 1), s0);
                } else {  // ServerKey::add (server_key.rs:89-102)
                    for (size_t i = 0; i < L; i++) R(i, clk) = fe_add(R(i, clk - 1), R(i + L, clk - 1));
                }
                for (size_t i = need; i < depth; i++) R(i - pos, clk) = R(i, clk - 1);  // shift_left
                for (size_t i = depth - pos; i < depth; i++) R(i, clk) = fe_zero();
                depth -= pos;
            }
            }
            helper[clk] = fe_make(depth);
            for (int i = 0; i < 5; i++) bits[i][clk - 1] = fe_make((o.code >> i) & 1);
            if (!rescue.is_round() && o.code != NOOP) {
                vm_err = "chiplets error at " + std::to_string(clk) + ": expected noop but was " + op_str(o);
                return ZK_ERR_CHIPLETS;
            }
            rescue.update(o.code, o.value);
            hflag[clk - 1] = fe_one();
            for (int i = 0; i < 4; i++) sponge[i][clk] = rescue.s[i];
        }
        if (clk % CYCLE) {
            vm_err = "chiplets error at " + std::to_string(clk) + ": trace length should be a multiple of 16, but was " +
                     std::to_string(clk);
            return ZK_ERR_CHIPLETS;
        }
        return ZK_OK;
    }

    size_t trace_len() const {
        size_t n = 1;
        while (n < cap + 1) n *= 2;
        return n;
    }

    void write(fe *t, size_t n, const fe *last) const {
        for (size_t r = 0; r < n; r++) {
            size_t rr = r <= clk ? r : clk;
            t[r] = fe_make(r);
            for (int i = 0; i < 5; i++) t[(1 + i) * n + r] = r <= clk ? bits[i][r] : fe_zero();
            t[6 * n + r] = r <= clk ? hflag[r] : fe_zero();
            for (int i = 0; i < 4; i++) t[(7 + i) * n + r] = sponge[i][rr];
            t[11 * n + r] = helper[rr];
            for (int i = 0; i < MAX_STACK; i++) t[(12 + i) * n + r] = reg[i][rr];
        }
        for (int c = 0; c < 28; c++) t[c * n + n - 1] = last[c];
    }
};

}  // namespace

extern "C" int zk_vm_trace(const char *source, const uint8_t *public_in, size_t num_public, const uint8_t *secret,
                           size_t num_secret, uint32_t lwe_size, uint32_t delta, const uint8_t *last_row,
                           uint8_t *trace_out, size_t cap_rows, size_t *n_out, uint8_t *outputs,
                           uint8_t *program_hash) {
    if (!source || !last_row || !n_out || lwe_size == 0 || lwe_size > 15 || (num_secret && !secret))
        return ZK_ERR_INVALID_ARG;
    std::vector<Op> code;
    int rc = compile(source, code);
    if (rc) return rc;
    if (!trace_out) {
        // size query: one clock per compiled op, so the length follows from the program alone
        // (Processor::grow doubles the capacity past clk; trace_len() is the next power of two above it)
        size_t cap = MIN_TRACE;
        while (code.size() >= cap) cap *= 2;
        size_t n = 1;
        while (n < cap + 1) n *= 2;
        *n_out = n;
        return ZK_ERR_BUFFER_TOO_SMALL;
    }
    std::vector<fe> sec(num_secret * lwe_size);
    for (size_t i = 0; i < sec.size(); i++) sec[i] = fe_from_bytes(secret + 16 * i);
    Processor P;
    rc = P.run(code, public_in, num_public, sec.data(), num_secret, lwe_size, delta);
    if (rc) return rc;
    size_t n = P.trace_len();
    *n_out = n;
    if (!trace_out || n > cap_rows) return ZK_ERR_BUFFER_TOO_SMALL;
    std::vector<fe> last(28);
    for (int c = 0; c < 28; c++) last[c] = fe_from_bytes(last_row + 16 * c);
    P.write(reinterpret_cast<fe *>(trace_out), n, last.data());
    if (outputs)
        for (int i = 0; i < MAX_STACK; i++) fe_to_bytes(P.reg[i][P.clk], outputs + 16 * i);
    if (program_hash) {  // Program::compile's hash = the chiplet's sponge after the whole program
        fe_to_bytes(P.rescue.s[0], program_hash);
        fe_to_bytes(P.rescue.s[1], program_hash + 16);
    }
    return ZK_OK;
}

extern "C" const char *zk_vm_last_error(void) { return vm_err.c_str(); }
