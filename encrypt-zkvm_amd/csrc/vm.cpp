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

#include <stdlib.h>

#include <algorithm>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zkvm_gpu.h"
#include "host_field.hpp"
#include "rescue_consts.hpp"
#include "vm_internal.hpp"

using namespace zk;
using namespace zk::vm;

namespace zk {
namespace vm {
thread_local std::string vm_err;
}
}  // namespace zk

namespace {

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

// a^2 (mod p) as any 128-bit representative (a itself may be one): fe_reduce_wide without the final
// conditional subtraction of p, which sits on the critical path of the squaring chains below; the
// multiplies that close each chain (fe_mul) return the canonical value.
inline fe sqr_lazy(fe a) {
    typedef unsigned __int128 u128;
    const u128 p00 = (u128)a.lo * a.lo, p01 = (u128)a.lo * a.hi, p11 = (u128)a.hi * a.hi;
    const u128 mid = (p00 >> 64) + (u128)(uint64_t)p01 * 2;
    const u128 lo = (mid << 64) | (uint64_t)p00;
    const u128 hi = p11 + (p01 >> 64) * 2 + (mid >> 64);
    const u128 t0 = (u128)(uint64_t)hi * ZK_C, t1 = (u128)(uint64_t)(hi >> 64) * ZK_C;
    const u128 s1 = lo + t0, s2 = s1 + (t1 << 64);
    const uint64_t top = (uint64_t)(t1 >> 64) + (uint64_t)(s1 < lo) + (uint64_t)(s2 < s1);
    u128 r = s2 + (u128)top * ZK_C;
    if (r < s2) r += ZK_C;
    return fe{(uint64_t)r, (uint64_t)(r >> 64)};
}

// The S-box chains of the four state elements are independent: each step below runs the four
// lanes back to back (lane loop innermost), which lets the out-of-order core overlap the four
// multiply chains (~4.4 ns per product instead of ~10 for one chain).
__attribute__((noinline)) void sqn4(fe v[4], int k) {  // v^(2^k), lazy representatives
    for (int t = 0; t < k; t++)
        for (int i = 0; i < 4; i++) v[i] = sqr_lazy(v[i]);
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

// ---------------------------------------------------------------- compiled program (Program::compile)
// The chiplet's sponge (columns 7-10 of the trace) absorbs (op code, op value) of every step and nothing else
// (vm/src/processor/chiplets.rs; crypto/src/rescue.rs:102-118): it is a function of the compiled code alone, and
// its final state is Program::compile's hash (vm/src/program/mod.rs:88-95).  The reference hashes the code at
// compile time and runs the same sponge again inside every Processor::run; here the compiled program keeps the
// per-step states it computed for the hash (CompiledProgram, vm_internal.hpp), so a run of the program on new
// inputs (the per-proof step) is the stack machine and the column writes only, split over threads.

int build_program(const char *source, CompiledProgram &P) {
    int rc = compile(source, P.code);
    if (rc) return rc;
    const size_t len = P.code.size();
    for (auto &v : P.sponge) v.resize(len + 1);
    for (int i = 0; i < 4; i++) P.sponge[i][0] = fe_zero();
    Rescue r;
    for (size_t k = 0; k < len; k++) {
        const Op o = P.code[k];
        if (!r.is_round() && o.code != NOOP && !P.chiplet_err) P.chiplet_err = k + 1;
        r.update(o.code, o.value);
        for (int i = 0; i < 4; i++) P.sponge[i][k + 1] = r.s[i];
    }
    P.hash[0] = r.s[0];
    P.hash[1] = r.s[1];
    // Processor::grow doubles the capacity past clk; trace_len() is the next power of two above it
    size_t cap = MIN_TRACE;
    while (len >= cap) cap *= 2;
    size_t n = 1;
    while (n < cap + 1) n *= 2;
    P.trace_len = n;
    return ZK_OK;
}

// ---------------------------------------------------------------- Processor::run -> trace
// The stack machine (vm/src/processor/stack.rs; the ciphertext ops of fhe/src/server_key.rs:89-124) on a small
// register file.  Pass 1 runs it once over the whole program, sequentially (each step reads the previous one),
// checks every error the reference raises and keeps the state at chunk boundaries; pass 2 replays the chunks on
// T threads, each writing its own rows of all 28 columns straight into the caller's column-major trace.
struct StackState {
    fe reg[MAX_STACK];
    size_t depth = 0, ta = 0, tb = 0;
};

struct Machine {
    const uint8_t *pub;
    size_t npub;
    const fe *sec;
    size_t nsec;
    uint32_t L, delta;

    // one step (clk is the 1-based step of op o, for the error texts); next := state after o
    int step(const StackState &cur, StackState &nx, Op o, size_t clk) const {
        auto stack_err = [&](const std::string &what) {
            vm_err = "stack error at " + std::to_string(clk) + ": " + what;
            return ZK_ERR_STACK;
        };
        nx.ta = cur.ta;
        nx.tb = cur.tb;
        size_t depth = cur.depth;
        switch (o.code) {
        case NOOP:
            for (size_t i = 0; i < depth; i++) nx.reg[i] = cur.reg[i];
            break;
        case PUSH:
        case READ:
        case READ2: {
            const size_t cnt = o.code == READ2 ? L : 1;
            if (o.code == READ2 && cur.tb >= nsec) return stack_err("no more inputs to " + op_str(o));
            depth += cnt;
            if (depth > (size_t)MAX_STACK) return stack_err(op_str(o) + " operation stack overflow");
            if (o.code == READ && cur.ta >= npub) return stack_err("no more inputs to " + op_str(o));
            for (size_t i = 0; i < depth - cnt; i++) nx.reg[i + cnt] = cur.reg[i];
            if (o.code == PUSH) nx.reg[0] = fe_make(o.value);
            else if (o.code == READ) nx.reg[0] = fe_make(pub[nx.ta++]);
            else {
                for (size_t i = 0; i < L; i++) nx.reg[i] = sec[cur.tb * L + i];
                nx.tb++;
            }
            break;
        }
        default: {
            const size_t need = (o.code == ADD || o.code == MUL) ? 2 : o.code == ADD2 ? 2 * L : L + 1;
            const size_t pos = o.code == ADD2 ? L : 1;
            if (depth < need) return stack_err(op_str(o) + " operation stack underflow");
            const fe s0 = cur.reg[0];
            if (o.code == ADD) nx.reg[0] = fe_add(s0, cur.reg[1]);
            else if (o.code == MUL) nx.reg[0] = fe_mul(s0, cur.reg[1]);
            else if (o.code == SADD) {  // ServerKey::scalar_add (fhe/src/server_key.rs:104-114)
                for (size_t i = 0; i < L; i++) {
                    fe v = cur.reg[1 + i];
                    if (i == L - 1) v = fe_add(v, fe_mul(fe_make(delta), s0));
                    nx.reg[i] = v;
                }
            } else if (o.code == SMUL) {  // ServerKey::scalar_mul (server_key.rs:116-124)
                for (size_t i = 0; i < L; i++) nx.reg[i] = fe_mul(cur.reg[1 + i], s0);
            } else {  // ServerKey::add (server_key.rs:89-102)
                for (size_t i = 0; i < L; i++) nx.reg[i] = fe_add(cur.reg[i], cur.reg[i + L]);
            }
            for (size_t i = need; i < depth; i++) nx.reg[i - pos] = cur.reg[i];  // shift_left
            for (size_t i = depth - pos; i < depth; i++) nx.reg[i] = fe_zero();
            depth -= pos;
        }
        }
        for (size_t i = depth; i < (size_t)MAX_STACK; i++) nx.reg[i] = fe_zero();
        nx.depth = depth;
        return ZK_OK;
    }
};

int vm_threads() {
    const char *e = getenv("ZK_VM_THREADS");
    if (!e) e = getenv("OMP_NUM_THREADS");
    int t = e ? atoi(e) : 0;
    if (t <= 0) t = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(t, 64));
}

// rows [r0, r1) of the trace: row r holds clk = r (column 0), the bits / hash flag of op r (r < len), and the
// sponge / depth / stack after step min(r, len); the last row is the caller's random row (processor/mod.rs:86-92)
void write_rows(const CompiledProgram &P, const Machine &M, StackState st, size_t r0, size_t r1, fe *t, size_t n,
                const fe *last) {
    const size_t len = P.code.size();
    StackState nx;
    for (size_t r = r0; r < r1; r++) {
        if (r == n - 1) {
            for (int c = 0; c < 28; c++) t[c * n + r] = last[c];
            continue;
        }
        if (r >= 1 && r <= len) {  // the state after step r
            (void)M.step(st, nx, P.code[r - 1], r);  // pass 1 already ran every step without error
            st = nx;
        }
        const size_t rr = r <= len ? r : len;
        const Op o = r < len ? P.code[r] : Op{NOOP, 0};
        t[r] = fe_make(r);
        for (int i = 0; i < 5; i++) t[(1 + i) * n + r] = fe_make(r < len ? (o.code >> i) & 1 : 0);
        t[6 * n + r] = r < len ? fe_one() : fe_zero();
        for (int i = 0; i < 4; i++) t[(7 + i) * n + r] = P.sponge[i][rr];
        t[11 * n + r] = fe_make(st.depth);
        for (int i = 0; i < MAX_STACK; i++) t[(12 + i) * n + r] = st.reg[i];
    }
}

// Pass 1 the reference's way (Machine::step, a full register copy per op): only to report the first error with the
// reference's status and text once the fast pass (stack_pass_impl) has found that the run fails.
int slow_pass_error(const CompiledProgram &P, const Machine &M) {
    const size_t len = P.code.size();
    StackState st, nx;
    for (size_t k = 1; k <= len; k++) {
        int rc = M.step(st, nx, P.code[k - 1], k);
        if (rc) return rc;
        st = nx;
        if (P.chiplet_err == k) {
            vm_err = "chiplets error at " + std::to_string(k) + ": expected noop but was " + op_str(P.code[k - 1]);
            return ZK_ERR_CHIPLETS;
        }
    }
    if (len % CYCLE) {
        vm_err = "chiplets error at " + std::to_string(len) + ": trace length should be a multiple of 16, but was " +
                 std::to_string(len);
        return ZK_ERR_CHIPLETS;
    }
    vm_err = "internal error: the VM's two stack passes disagree";
    return ZK_ERR_INVALID_ARG;
}

// The stack pass (vm_internal.hpp stack_pass): states[c] = the state row row_of(c) - 1 shows.  The stack is kept
// bottom first (b[0..d)), so a push is one store, a pop a decrement and the ciphertext ops touch their L slots only.
// LT: the ciphertext width L as a compile-time constant (1 .. 5, the ciphertext loops unrolled), or 0 (in.L).
template <int LT, class RowOf>
int stack_pass_run(const CompiledProgram &P, const Inputs &in, size_t nstates, RowOf row_of, VmState *states,
                   fe *outputs, uint32_t *max_depth) {
    const size_t len = P.code.size(), L = LT ? (size_t)LT : in.L;
    const fe delta = fe_make(in.delta);
    fe b[MAX_STACK];
    size_t d = 0, ta = 0, tb = 0, c = 0, md = 0;
    auto snap = [&](VmState &s) {
        for (size_t i = 0; i < (size_t)MAX_STACK; i++) s.reg[i] = i < d ? b[d - 1 - i] : fe_zero();
        s.depth = (uint32_t)d;
        s.ta = (uint32_t)ta;
        s.tb = (uint32_t)tb;
        s.pad = 0;
    };
    auto sec = [&](size_t i) { return fe_from_bytes(in.sec + 16 * i); };
    while (c < nstates && row_of(c) <= 1) snap(states[c++]);  // rows -1 and 0 show the zero state
    size_t next = c < nstates ? row_of(c) : SIZE_MAX;  // the row of the next state to keep
    bool err = false;
    for (size_t k = 1; k <= len && !err; k++) {
        const Op o = P.code[k - 1];
        switch (o.code) {
        case NOOP:
            break;
        case PUSH:
            if (d + 1 > (size_t)MAX_STACK) err = true;
            else b[d++] = fe_make(o.value);
            break;
        case READ:
            if (d + 1 > (size_t)MAX_STACK || ta >= in.npub) err = true;
            else b[d++] = fe_make(in.pub[ta++]);
            break;
        case READ2:
            if (tb >= in.nsec || d + L > (size_t)MAX_STACK) err = true;
            else {
                for (size_t i = 0; i < L; i++) b[d + L - 1 - i] = sec(tb * L + i);
                d += L;
                tb++;
            }
            break;
        case ADD:
        case MUL:
            if (d < 2) err = true;
            else {
                b[d - 2] = o.code == ADD ? fe_add(b[d - 1], b[d - 2]) : fe_mul(b[d - 1], b[d - 2]);
                d--;
            }
            break;
        case SADD:  // ServerKey::scalar_add (fhe/src/server_key.rs:104-114): s'[L-1] = s[L] + delta s0
            if (d < L + 1) err = true;
            else {
                const fe s0 = b[--d];
                b[d - L] = fe_add(b[d - L], fe_mul(delta, s0));
            }
            break;
        case SMUL:  // ServerKey::scalar_mul (server_key.rs:116-124): s'[i] = s[i + 1] s0
            if (d < L + 1) err = true;
            else {
                const fe s0 = b[--d];
                for (size_t i = 0; i < L; i++) b[d - 1 - i] = fe_mul(b[d - 1 - i], s0);
            }
            break;
        case ADD2:  // ServerKey::add (server_key.rs:89-102): s'[i] = s[i] + s[i + L]
            if (d < 2 * L) err = true;
            else {
                for (size_t i = 0; i < L; i++) b[d - L - 1 - i] = fe_add(b[d - 1 - i], b[d - L - 1 - i]);
                d -= L;
            }
            break;
        default:
            err = true;
        }
        if (P.chiplet_err == k) err = true;
        md = std::max(md, d);
        if (k + 1 == next && !err) {
            do
                snap(states[c++]);
            while (c < nstates && row_of(c) == k + 1);
            next = c < nstates ? row_of(c) : SIZE_MAX;
        }
    }
    if (err || len % CYCLE) {
        std::vector<fe> sv(in.nsec * L);
        for (size_t i = 0; i < sv.size(); i++) sv[i] = sec(i);
        return slow_pass_error(P, Machine{in.pub, in.npub, sv.data(), in.nsec, in.L, in.delta});
    }
    while (c < nstates) snap(states[c++]);
    if (max_depth) *max_depth = (uint32_t)md;
    if (outputs)
        for (size_t i = 0; i < (size_t)MAX_STACK; i++) outputs[i] = i < d ? b[d - 1 - i] : fe_zero();
    return ZK_OK;
}
template <class RowOf>
int stack_pass_impl(const CompiledProgram &P, const Inputs &in, size_t nstates, RowOf row_of, VmState *states,
                    fe *outputs, uint32_t *max_depth = nullptr) {
    switch (in.L) {
    case 1: return stack_pass_run<1>(P, in, nstates, row_of, states, outputs, max_depth);
    case 2: return stack_pass_run<2>(P, in, nstates, row_of, states, outputs, max_depth);
    case 3: return stack_pass_run<3>(P, in, nstates, row_of, states, outputs, max_depth);
    case 4: return stack_pass_run<4>(P, in, nstates, row_of, states, outputs, max_depth);
    case 5: return stack_pass_run<5>(P, in, nstates, row_of, states, outputs, max_depth);
    default: return stack_pass_run<0>(P, in, nstates, row_of, states, outputs, max_depth);
    }
}

int run_program(const CompiledProgram &P, const Inputs &in, fe *t, size_t n, const fe *last, fe *outputs) {
    const int T = (int)std::min<size_t>((size_t)vm_threads(), std::max<size_t>(1, n / 4096));
    // chunk c covers rows [bnd[c], bnd[c + 1]) and starts from the state row bnd[c] - 1 shows (write_rows steps
    // once before writing a row in [1, len]; chunk 0 starts from the zero state at row 0)
    std::vector<size_t> bnd(T + 1);
    for (int c = 0; c <= T; c++) bnd[c] = n * (size_t)c / (size_t)T;
    std::vector<VmState> vs(T);
    int rc = stack_pass_impl(P, in, (size_t)T, [&](size_t c) { return bnd[c]; }, vs.data(), outputs);
    if (rc || !t) return rc;
    std::vector<fe> sec(in.nsec * in.L);
    for (size_t i = 0; i < sec.size(); i++) sec[i] = fe_from_bytes(in.sec + 16 * i);
    const Machine M{in.pub, in.npub, sec.data(), in.nsec, in.L, in.delta};
    std::vector<StackState> start(T);
    for (int c = 0; c < T; c++) {
        memcpy(start[c].reg, vs[c].reg, sizeof start[c].reg);
        start[c].depth = vs[c].depth;
        start[c].ta = vs[c].ta;
        start[c].tb = vs[c].tb;
    }
    // a thread that cannot be started (resource limits) leaves its chunk to the calling thread: no exception may
    // cross the C ABI
    std::vector<std::thread> th;
    std::vector<int> mine;
    for (int k = 1; k < T; k++) {
        try {
            th.emplace_back(write_rows, std::cref(P), std::cref(M), start[k], bnd[k], bnd[k + 1], t, n, last);
        } catch (...) {
            mine.push_back(k);
        }
    }
    write_rows(P, M, StackState(), 0, bnd[1], t, n, last);
    for (int k : mine) write_rows(P, M, start[k], bnd[k], bnd[k + 1], t, n, last);
    for (auto &x : th) x.join();
    return ZK_OK;
}

}  // namespace

int zk::vm::stack_pass(const CompiledProgram &P, const Inputs &in, size_t stride, size_t nstates, VmState *states,
                       fe *outputs, uint32_t *max_depth) {
    return stack_pass_impl(P, in, nstates, [stride](size_t c) { return c * stride; }, states, outputs, max_depth);
}

extern "C" int zk_program_compile(const char *source, zk_program **out, uint8_t *program_hash, size_t *trace_len) {
    if (!source || !out) return ZK_ERR_INVALID_ARG;
    *out = nullptr;
    auto prog = std::make_unique<zk_program>();
    const int rc = build_program(source, prog->P);
    if (rc) return rc;
    if (program_hash) {
        fe_to_bytes(prog->P.hash[0], program_hash);
        fe_to_bytes(prog->P.hash[1], program_hash + 16);
    }
    if (trace_len) *trace_len = prog->P.trace_len;
    *out = prog.release();
    return ZK_OK;
}

extern "C" void zk_program_free(zk_program *prog) { delete prog; }

extern "C" int zk_program_trace(const zk_program *prog, const uint8_t *public_in, size_t num_public,
                                const uint8_t *secret, size_t num_secret, uint32_t lwe_size, uint32_t delta,
                                const uint8_t *last_row, uint8_t *trace_out, size_t cap_rows, size_t *n_out,
                                uint8_t *outputs) {
    if (!prog || !last_row || !n_out || lwe_size == 0 || lwe_size > 15 || (num_secret && !secret) ||
        (num_public && !public_in))
        return ZK_ERR_INVALID_ARG;
    const CompiledProgram &P = prog->P;
    const size_t n = P.trace_len;
    *n_out = n;
    if (trace_out && n > cap_rows) return ZK_ERR_BUFFER_TOO_SMALL;
    const Inputs in{public_in, num_public, secret, num_secret, lwe_size, delta};
    fe last[28], outs[MAX_STACK];
    for (int c = 0; c < 28; c++) last[c] = fe_from_bytes(last_row + 16 * c);
    const int rc = run_program(P, in, reinterpret_cast<fe *>(trace_out), n, last, outs);
    if (rc) return rc;
    if (outputs)
        for (int i = 0; i < MAX_STACK; i++) fe_to_bytes(outs[i], outputs + 16 * i);
    return trace_out ? ZK_OK : ZK_ERR_BUFFER_TOO_SMALL;
}

extern "C" int zk_vm_trace(const char *source, const uint8_t *public_in, size_t num_public, const uint8_t *secret,
                           size_t num_secret, uint32_t lwe_size, uint32_t delta, const uint8_t *last_row,
                           uint8_t *trace_out, size_t cap_rows, size_t *n_out, uint8_t *outputs,
                           uint8_t *program_hash) {
    if (!source || !last_row || !n_out || lwe_size == 0 || lwe_size > 15 || (num_secret && !secret))
        return ZK_ERR_INVALID_ARG;
    if (!trace_out) {
        // size query: one clock per compiled op, so the length follows from the program alone
        std::vector<Op> code;
        const int rc = compile(source, code);
        if (rc) return rc;
        size_t cap = MIN_TRACE;
        while (code.size() >= cap) cap *= 2;
        size_t n = 1;
        while (n < cap + 1) n *= 2;
        *n_out = n;
        return ZK_ERR_BUFFER_TOO_SMALL;
    }
    zk_program *prog = nullptr;
    int rc = zk_program_compile(source, &prog, program_hash, nullptr);
    if (rc) return rc;
    rc = zk_program_trace(prog, public_in, num_public, secret, num_secret, lwe_size, delta, last_row, trace_out,
                          cap_rows, n_out, outputs);
    zk_program_free(prog);
    return rc;
}

extern "C" const char *zk_vm_last_error(void) { return vm_err.c_str(); }
