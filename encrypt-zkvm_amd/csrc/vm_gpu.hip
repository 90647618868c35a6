// vm_gpu.hip -- the VM's trace written on the GPU, straight into the prover's trace buffer, and vm::prove as one call.
//
// The reference builds the 28-column trace on the host (Processor::run + trace, vm/src/processor/mod.rs:61-95)
// and hands it to Prover::prove (vm/src/lib.rs:13-29); moving it to the device costs 448 MiB over PCIe per
// 2^20-step proof.  Here the host keeps only the sequential part -- one pass of the stack machine, which checks every
// error the reference raises and produces the outputs (vm.cpp stack_pass) -- and ships the machine state every S rows
// plus the inputs (~6 MB at 2^20).  The GPU then:
//   k_vm_fixed   the 11 columns that do not depend on the inputs: clk, the 5 opcode bits, the hash flag, the sponge
//                state (from the program's device copy, uploaded once per device) and the last (random) row;
//   k_vm_states  one thread per S-row segment replays the stack machine from its coarse state and stores the state
//                every K rows (SoA, so the next kernel loads it coalesced);
//   k_vm_rows    one thread per K-row chunk replays K steps and writes the depth and the 16 stack registers of each
//                row (a lane's K consecutive rows fill whole 128-byte lines of each column).
// The device step is the reference's stack.rs semantics on a register file, top first, with static shifts: the
// ciphertext width L = lwe_size is a template parameter (1..5: the AIR's range, zk_prove's lwe_size check), so every
// shift is a fixed register move under the op's exec mask.
#include <hip/hip_runtime.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "comm.hpp"
#include "prover_internal.hpp"
#include "vm_internal.hpp"

using namespace zk;
using zk::vm::Op;
using zk::vm::VmState;

namespace {

constexpr int VM_S = 64;  // rows per host state (k_vm_states segment; ZK_VM_SEG overrides, a multiple of VM_K)
constexpr int VM_K = 8;   // rows per device state (k_vm_rows chunk)
constexpr int NREG = zk::vm::MAX_STACK;

struct DevState {
    fe t[NREG];
    uint32_t d, ta, tb;
};

template <int S>
__device__ __forceinline__ void shift_up(fe (&t)[NREG]) {  // t[i] = t[i - S]; t[0..S) are overwritten by the caller
#pragma unroll
    for (int i = NREG - 1; i >= S; i--) t[i] = t[i - S];
}
template <int S>
__device__ __forceinline__ void shift_down(fe (&t)[NREG]) {  // t[i] = t[i + S], zeros enter at the bottom
#pragma unroll
    for (int i = 0; i < NREG - S; i++) t[i] = t[i + S];
#pragma unroll
    for (int i = NREG - S; i < NREG; i++) t[i] = fe_zero();
}

// One op (vm/src/processor/stack.rs; the ciphertext ops of fhe/src/server_key.rs:89-124).  The host pass has run
// the program without error, so no check is repeated here; entries at or beyond the depth stay zero.
template <int L>
__device__ __forceinline__ void vm_step(DevState &s, Op o, const uint8_t *pub, const fe *sec, fe delta) {
    switch (o.code) {
    case zk::vm::PUSH:
    case zk::vm::READ: {
        const fe v = fe_make(o.code == zk::vm::PUSH ? o.value : pub[s.ta]);
        s.ta += o.code == zk::vm::READ;
        shift_up<1>(s.t);
        s.t[0] = v;
        s.d += 1;
        break;
    }
    case zk::vm::READ2: {
        shift_up<L>(s.t);
        const fe *c = sec + (size_t)s.tb * L;
#pragma unroll
        for (int i = 0; i < L; i++) s.t[i] = c[i];
        s.tb += 1;
        s.d += L;
        break;
    }
    case zk::vm::ADD:
    case zk::vm::MUL: {
        const fe v = o.code == zk::vm::ADD ? fe_add(s.t[0], s.t[1]) : fe_mul(s.t[0], s.t[1]);
        shift_down<1>(s.t);
        s.t[0] = v;
        s.d -= 1;
        break;
    }
    case zk::vm::SADD: {  // s'[i] = s[i + 1], s'[L - 1] += delta s0
        const fe s0 = s.t[0];
        shift_down<1>(s.t);
        s.t[L - 1] = fe_add(s.t[L - 1], fe_mul(delta, s0));
        s.d -= 1;
        break;
    }
    case zk::vm::SMUL: {  // s'[i] = s[i + 1] s0, i < L
        const fe s0 = s.t[0];
        shift_down<1>(s.t);
#pragma unroll
        for (int i = 0; i < L; i++) s.t[i] = fe_mul(s.t[i], s0);
        s.d -= 1;
        break;
    }
    case zk::vm::ADD2: {  // s'[i] = s[i] + s[i + L], i < L
#pragma unroll
        for (int i = 0; i < L; i++) s.t[i + L] = fe_add(s.t[i], s.t[i + L]);
        shift_down<L>(s.t);
        s.d -= L;
        break;
    }
    default:  // NOOP
        break;
    }
}

// SoA state planes: register i of state c at F[i * nf + c], {d, ta, tb} at F[NREG * nf + c]
__device__ __forceinline__ void store_state(fe *F, size_t nf, size_t c, const DevState &s) {
#pragma unroll
    for (int i = 0; i < NREG; i++) F[(size_t)i * nf + c] = s.t[i];
    reinterpret_cast<uint4 *>(F + (size_t)NREG * nf)[c] = make_uint4(s.d, s.ta, s.tb, 0);
}
__device__ __forceinline__ void load_state(const fe *F, size_t nf, size_t c, DevState &s) {
#pragma unroll
    for (int i = 0; i < NREG; i++) s.t[i] = F[(size_t)i * nf + c];
    const uint4 m = reinterpret_cast<const uint4 *>(F + (size_t)NREG * nf)[c];
    s.d = m.x;
    s.ta = m.y;
    s.tb = m.z;
}

// rows [t S, (t + 1) S): from the host's state of row t S - 1, the state of row c K - 1 for every chunk c inside
template <int L>
__global__ void __launch_bounds__(64) k_vm_states(const VmState *H, size_t nseg, int seg, const Op *code, size_t len,
                                                  const uint8_t *pub, const fe *sec, fe delta, fe *F, size_t nf) {
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= nseg) return;
    DevState s;
    const VmState &h = H[t];
#pragma unroll
    for (int i = 0; i < NREG; i++) s.t[i] = h.reg[i];
    s.d = h.depth;
    s.ta = h.ta;
    s.tb = h.tb;
    const size_t r0 = t * (size_t)seg;
    for (int k = 0;; k++) {
        const size_t r = r0 + k;
        if (k % VM_K == 0) {
            store_state(F, nf, r / VM_K, s);  // the state row r - 1 shows
            if (k == seg - VM_K) break;        // the next segment starts from the host's state
        }
        if (r >= 1 && r <= len) vm_step<L>(s, code[r - 1], pub, sec, delta);
    }
}

// rows [c K, (c + 1) K) of the machine's columns: the state after step min(r, len) of each row r -- the depth (column
// 11) when `depth`, the stack registers 0 .. nregs - 1 (columns 12 .. 12 + nregs - 1); row n - 1 holds the caller's
// random row, written here when `last` is given (else by k_vm_fixed)
template <int L>
__global__ void __launch_bounds__(256) k_vm_rows(const fe *F, size_t nf, const Op *code, size_t len,
                                                 const uint8_t *pub, const fe *sec, fe delta, int nregs, bool depth,
                                                 const fe *last, fe *trace, size_t n) {
    const size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (c >= nf) return;
    DevState s;
    load_state(F, nf, c, s);
    for (int k = 0; k < VM_K; k++) {
        const size_t r = c * VM_K + k;
        if (r == n - 1) {
            if (last)
                for (int i = 0; i < nregs; i++) trace[(size_t)(12 + i) * n + r] = last[12 + i];
            break;
        }
        if (r >= 1 && r <= len) vm_step<L>(s, code[r - 1], pub, sec, delta);
        if (depth) trace[11 * n + r] = fe_make(s.d);
#pragma unroll
        for (int i = 0; i < NREG; i++)
            if (i < nregs) trace[(size_t)(12 + i) * n + r] = s.t[i];
    }
}

// the input-independent columns: clk, opcode bits (col 5 = MSB), hash flag, sponge after step min(r, len); row n - 1
// is the caller's random row in every column (vm/src/processor/mod.rs:86-92)
__global__ void __launch_bounds__(256) k_vm_fixed(const Op *code, size_t len, const fe *sponge, const fe *last,
                                                  fe *trace, size_t n) {
    const size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (r >= n) return;
    if (r == n - 1) {
        for (int col = 0; col < 28; col++) trace[(size_t)col * n + r] = last[col];
        return;
    }
    const uint32_t op = r < len ? code[r].code : 0u;
    trace[r] = fe_make(r);
#pragma unroll
    for (int i = 0; i < 5; i++) trace[(size_t)(1 + i) * n + r] = fe_make((op >> i) & 1u);
    trace[6 * n + r] = fe_make(r < len ? 1u : 0u);
    const size_t rr = r <= len ? r : len;
#pragma unroll
    for (int i = 0; i < 4; i++) trace[(size_t)(7 + i) * n + r] = sponge[(size_t)i * (len + 1) + rr];
}

// the preprocessed columns (FixedCols): out[c][i] = F[src][i] (0 when src < 0) + last[c] base[i] for the ncol
// columns listed, over `count` points of planes of `stride` (coefficients: n; LDE: B n).  Streaming, HBM-bound: per
// point the Lagrange value once, then per column one read (nonzero f_c) and one write.
struct AxpyCols {
    int ncol;
    uint8_t col[W];
    int8_t src[W];
};
__global__ void __launch_bounds__(256) k_fixed_axpy(const fe *F, const fe *base, size_t stride, AxpyCols A,
                                                    const fe_ws *ws, fe *out) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= stride) return;
    const fe b = base[i];
#pragma unroll
    for (int k = 0; k < W; k++) {
        if (k < A.ncol) {
            const int c = A.col[k], s = A.src[k];
            const fe t = fe_mul_uniform(b, load_fe_ws(ws, c));
            out[(size_t)c * stride + i] = s >= 0 ? fe_add(F[(size_t)s * stride + i], t) : t;
        }
    }
}

template <int L>
void launch_machine(hipStream_t st, const VmState *H, size_t nseg, int seg, const Op *code, size_t len,
                    const uint8_t *pub, const fe *sec, fe delta, fe *F, size_t nf, int nregs, bool depth,
                    const fe *last, fe *trace, size_t n) {
    ZK_PROF(st, "vm_states", (double)nseg * sizeof(VmState) + (double)nf * (NREG + 1) * 16,
            hipLaunchKernelGGL(k_vm_states<L>, dim3((unsigned)((nseg + 63) / 64)), dim3(64), 0, st, H, nseg, seg, code,
                               len, pub, sec, delta, F, nf));
    ZK_PROF(st, "vm_rows", (double)nf * (NREG + 1) * 16 + (double)n * (nregs + depth) * 16,
            hipLaunchKernelGGL(k_vm_rows<L>, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, st, F, nf, code, len,
                               pub, sec, delta, nregs, depth, last, trace, n));
}

struct DevProg {
    const Op *code;
    const fe *sponge;
};

// the program's code and sponge columns on `device` (uploaded once, kept until zk_program_free); prog->mu held
int device_program_locked(zk_program *prog, int device, zk_program::Device **out) {
    for (auto &d : prog->dev)
        if (d->device == device) {
            *out = d.get();
            return ZK_OK;
        }
    const auto &P = prog->P;
    const size_t len = P.code.size();
    auto d = std::make_unique<zk_program::Device>();
    d->device = device;
    d->code = nullptr;
    d->sponge = nullptr;
    ZK_CHECK_HIP(hipMalloc(&d->code, len * sizeof(Op) + 16));
    zk_program::Device *raw = d.get();
    prog->dev.push_back(std::move(d));  // freed by ~zk_program even if a step below fails
    ZK_CHECK_HIP(hipMalloc(&raw->sponge, 4 * (len + 1) * sizeof(fe)));
    ZK_CHECK_HIP(hipMemcpy(raw->code, P.code.data(), len * sizeof(Op), hipMemcpyHostToDevice));
    for (int i = 0; i < 4; i++)
        ZK_CHECK_HIP(hipMemcpy(raw->sponge + (size_t)i * (len + 1), P.sponge[i].data(), (len + 1) * sizeof(fe),
                               hipMemcpyHostToDevice));
    *out = raw;
    return ZK_OK;
}

int device_program(zk_program *prog, int device, DevProg *out) {
    std::lock_guard<std::mutex> lk(prog->mu);
    zk_program::Device *d = nullptr;
    ZK_TRY(device_program_locked(prog, device, &d));
    *out = DevProg{d->code, d->sponge};
    return ZK_OK;
}

// Processor::trace's random last row (vm/src/processor/mod.rs:86-92: a nonzero u128 that is a field element)
void random_last_row(fe last[28]) {
    std::random_device rd;
    for (int c = 0; c < 28; c++) {
        for (;;) {
            const uint64_t lo = ((uint64_t)rd() << 32) | rd(), hi = ((uint64_t)rd() << 32) | rd();
            const bool below_p = hi < ZK_P_HI || (hi == ZK_P_HI && lo < ZK_P_LO);
            if (below_p && (lo | hi)) {
                last[c] = fe_make(lo, hi);
                break;
            }
        }
    }
}

// Which columns of the trace vm_generate writes
struct GenMode {
    bool fixed;  // the input-independent columns 0..10 and the depth (11)
    int nregs;   // stack registers 0 .. nregs - 1 (columns 12 ..)
};

// The trace of `prog` on `in` into p->d_trace (28 x n column-major; the columns `mode` selects), stream-ordered on
// p->st: the host stack pass (errors, outputs, the state every S rows, the maximum depth), one upload of the states,
// inputs and last row, then the kernels.  Nothing waits for them.
// dp_known: the program's device copy when the caller holds prog->mu (fixed_columns), else null (looked up here)
int vm_generate(zk_prover *p, zk_program *prog, const zk::vm::Inputs &in, const fe last[28], GenMode mode,
                size_t *n_out, fe *outputs, uint32_t *max_depth, const DevProg *dp_known = nullptr) {
    const auto &P = prog->P;
    const size_t n = P.trace_len, len = P.code.size();
    *n_out = n;
    if (n > p->max_n) ZK_FAIL(ZK_ERR_INVALID_ARG, "the program's trace is longer than the prover's max_trace_len");
    if (in.L < 1 || in.L > 5)
        ZK_FAIL(ZK_ERR_INVALID_ARG, "lwe_size must be in [1, 5] (the AIR's ciphertext width, as zk_prove requires)");
    ZK_CHECK_HIP(hipSetDevice(p->device));
    static const size_t seg_env = [] {
        const char *e = getenv("ZK_VM_SEG");
        const long v = e ? atol(e) : 0;
        return (v >= VM_K && v % VM_K == 0 && v <= 4096) ? (size_t)v : (size_t)VM_S;
    }();
    const size_t S = std::min<size_t>(seg_env, n), nseg = n / S, nf = n / VM_K;
    // the staging area is reused: the previous upload from it must have completed (an event, not a stream sync: the
    // stream may hold zk_vm_prove's preprocessed-column work, which runs while this host pass does)
    if (p->ev_vm_live) ZK_CHECK_HIP(hipEventSynchronize(p->ev_vm));
    p->ev_vm_live = false;
    if (!p->ev_vm) ZK_CHECK_HIP(hipEventCreateWithFlags(&p->ev_vm, hipEventDisableTiming));
    const size_t b_states = nseg * sizeof(VmState), b_sec = in.nsec * in.L * sizeof(fe), b_last = 28 * sizeof(fe);
    const size_t bytes = b_states + b_sec + b_last + in.npub;
    if (bytes > 8 * p->max_n * sizeof(fe)) ZK_FAIL(ZK_ERR_INVALID_ARG, "too many inputs for the prover's staging area");
    if (bytes + 64 > p->h_vm_cap) {
        if (p->h_vm) (void)hipHostFree(p->h_vm);
        p->h_vm = nullptr;
        p->h_vm_cap = 0;
        ZK_CHECK_HIP(hipHostMalloc((void **)&p->h_vm, bytes + 64, hipHostMallocDefault));
        p->h_vm_cap = bytes + 64;
    }
    uint8_t *h = p->h_vm;
    // the sequential part on the host: every error the reference raises, the outputs, the state every S rows
    const int rc = zk::vm::stack_pass(P, in, S, nseg, reinterpret_cast<VmState *>(h), outputs, max_depth);
    if (rc) {
        g_err = zk::vm::vm_err;
        return rc;
    }
    if (b_sec) memcpy(h + b_states, in.sec, b_sec);
    memcpy(h + b_states + b_sec, last, b_last);
    if (in.npub) memcpy(h + b_states + b_sec + b_last, in.pub, in.npub);
    DevProg dp;
    if (dp_known) dp = *dp_known;
    else ZK_TRY(device_program(prog, p->device, &dp));
    // device staging: the composition scratch (8 n elements, free until the composition step) holds the upload, the
    // NTT scratch the device states; neither is touched by the preprocessed columns' work queued before this pass
    uint8_t *dv = reinterpret_cast<uint8_t *>(p->ctmp);
    ZK_CHECK_HIP(hipMemcpyAsync(dv, h, bytes, hipMemcpyHostToDevice, p->st));
    ZK_CHECK_HIP(hipEventRecord(p->ev_vm, p->st));
    p->ev_vm_live = true;
    const VmState *dH = reinterpret_cast<const VmState *>(dv);
    const fe *dsec = reinterpret_cast<const fe *>(dv + b_states);
    const fe *dlast = reinterpret_cast<const fe *>(dv + b_states + b_sec);
    const uint8_t *dpub = dv + b_states + b_sec + b_last;
    fe *F = p->tmp;
    const fe dl = fe_make(in.delta);
    if (mode.fixed)
        ZK_PROF(p->st, "vm_fixed", (double)n * 11 * 16,
                hipLaunchKernelGGL(k_vm_fixed, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, p->st, dp.code, len,
                                   dp.sponge, dlast, p->d_trace, n));
    const fe *rlast = mode.fixed ? nullptr : dlast;
#define ZK_VM_LAUNCH(LL)                                                                                              \
    launch_machine<LL>(p->st, dH, nseg, (int)S, dp.code, len, dpub, dsec, dl, F, nf, mode.nregs, mode.fixed, rlast, \
                       p->d_trace, n)
    switch (in.L) {
    case 1: ZK_VM_LAUNCH(1); break;
    case 2: ZK_VM_LAUNCH(2); break;
    case 3: ZK_VM_LAUNCH(3); break;
    case 4: ZK_VM_LAUNCH(4); break;
    default: ZK_VM_LAUNCH(5); break;
    }
#undef ZK_VM_LAUNCH
    ZK_CHECK_HIP(hipGetLastError());
    return ZK_OK;
}

// The preprocessed columns of (prog, lwe_size, blowup) on p's device (zk_program::Fixed), built on first use with
// this call's inputs: the full trace with a zero last row, its columns 0..11 interpolated and extended, and the
// Lagrange polynomial of the last row.  Returned by value (the cache may grow while the caller proves).
// r0, ncos: the LDE cosets to hold (a sharded rank's block r0 .. r0 + ncos - 1; 0, 0 for all B of them).
int fixed_columns(zk_prover *p, zk_program *prog, const zk::vm::Inputs &in, uint32_t B, zk_program::Fixed *out,
                  int r0 = 0, int ncos = 0) {
    if (!ncos) ncos = (int)B;
    std::lock_guard<std::mutex> lk(prog->mu);
    zk_program::Device *d = nullptr;
    ZK_TRY(device_program_locked(prog, p->device, &d));
    for (const auto &f : d->fixed)
        if (f.L == in.L && f.B == B && f.r0 == r0 && f.ncos == ncos) {
            *out = f;
            return ZK_OK;
        }
    const size_t n = prog->P.trace_len;
    const uint32_t nb = (uint32_t)ncos;  // cosets held
    Plan *pl = nullptr;
    ZK_TRY(get_plan(p, n, B, &pl));
    // built in a local entry and cached only once complete: a call whose inputs the VM refuses (too few inputs, ...)
    // leaves no half-built entry behind for the program's later calls
    zk_program::Fixed g{in.L, B, 0, nullptr, nullptr, nullptr, nullptr, r0, ncos};
    struct Unwind {
        zk_program::Fixed *g;
        ~Unwind() {
            if (!g) return;
            (void)hipFree(g->fpolys);
            (void)hipFree(g->flde);
            (void)hipFree(g->lagr);
            (void)hipFree(g->lagr_lde);
        }
    } unwind{&g};
    ZK_CHECK_HIP(hipMalloc(&g.fpolys, 12 * n * sizeof(fe)));
    ZK_CHECK_HIP(hipMalloc(&g.flde, 12 * nb * n * sizeof(fe)));
    ZK_CHECK_HIP(hipMalloc(&g.lagr, n * sizeof(fe)));
    ZK_CHECK_HIP(hipMalloc(&g.lagr_lde, nb * n * sizeof(fe)));
    // f_0 .. f_11: the program-only columns with the last row zeroed
    fe zero[28], outs[NREG];
    memset(zero, 0, sizeof zero);
    uint32_t md = 0;
    size_t nn = 0;
    const DevProg dp{d->code, d->sponge};  // prog->mu is held: no second lookup through device_program
    ZK_TRY(vm_generate(p, prog, in, zero, GenMode{true, NREG}, &nn, outs, &md, &dp));
    const fe inv_n = h_inv(fe_make(n));
    ntt(p->st, pl->Tn, p->d_trace, n, g.fpolys, n, 12, true, nullptr, &inv_n, p->tmp);
    ntt_lde(p->st, pl->Tn, pl->ct, g.fpolys, n, 12, r0, 1, (int)nb, g.flde, nb * n, n, p->tmp);
    // e_(n-1): zeros but a one in the last row
    ZK_CHECK_HIP(hipMemsetAsync(p->polys, 0, n * sizeof(fe), p->st));
    const fe one = fe_one();
    ZK_TRY(h2d_small(p, p->polys + (n - 1), &one, sizeof one));
    ntt(p->st, pl->Tn, p->polys, n, g.lagr, n, 1, true, nullptr, &inv_n, p->tmp);
    ntt_lde(p->st, pl->Tn, pl->ct, g.lagr, n, 1, r0, 1, (int)nb, g.lagr_lde, nb * n, n, p->tmp);
    ZK_TRY(io_rewind(p));  // sync: the cache is complete, the staging area starts over
    g.md = (int)md;
    d->fixed.push_back(g);  // freed by ~zk_program from here on
    unwind.g = nullptr;
    *out = g;
    return ZK_OK;
}

}  // namespace

void zk::fixed_axpy(hipStream_t st, const FixedCols &fx, const fe_ws *ws_dev, size_t n, size_t B, fe *polys, fe *lde) {
    AxpyCols A;
    A.ncol = 0;
    for (int c = 0; c < W; c++) {
        if (c >= 12 && c < 12 + fx.md) continue;  // dynamic: interpolated and extended from the trace
        A.col[A.ncol] = (uint8_t)c;
        A.src[A.ncol] = (int8_t)(c < 12 ? c : -1);
        A.ncol++;
    }
    const size_t nf = 12, nz = (size_t)A.ncol - nf;
    ZK_PROF(st, "fixed_axpy", (double)n * 16 * (1 + 2 * nf + nz),
            hipLaunchKernelGGL(k_fixed_axpy, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, fx.fpolys, fx.lagr, n, A,
                               ws_dev, polys));
    ZK_PROF(st, "fixed_axpy", (double)B * n * 16 * (1 + 2 * nf + nz),
            hipLaunchKernelGGL(k_fixed_axpy, dim3((unsigned)((B * n + 255) / 256)), dim3(256), 0, st, fx.flde,
                               fx.lagr_lde, B * n, A, ws_dev, lde));
}

zk_program::~zk_program() {
    for (auto &d : dev) {
        (void)hipSetDevice(d->device);
        (void)hipFree(d->code);
        (void)hipFree(d->sponge);
        for (auto &f : d->fixed) {
            (void)hipFree(f.fpolys);
            (void)hipFree(f.flde);
            (void)hipFree(f.lagr);
            (void)hipFree(f.lagr_lde);
        }
    }
}

static void read_last(const uint8_t *last_row, fe last[28]) {
    if (last_row)
        for (int c = 0; c < 28; c++) last[c] = fe_from_bytes(last_row + 16 * c);
    else
        random_last_row(last);
}

int zk_vm_trace_device(zk_prover *p, zk_program *prog, const uint8_t *public_in, size_t num_public,
                       const uint8_t *secret, size_t num_secret, uint32_t lwe_size, uint32_t delta,
                       const uint8_t *last_row, size_t *n_out, uint8_t *outputs) {
    if (!p || !prog || !n_out || (num_secret && !secret) || (num_public && !public_in))
        ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    fe outs[NREG], last[28];
    read_last(last_row, last);
    const zk::vm::Inputs in{public_in, num_public, secret, num_secret, lwe_size, delta};
    ZK_TRY(vm_generate(p, prog, in, last, GenMode{true, NREG}, n_out, outs, nullptr));
    ZK_CHECK_HIP(hipStreamSynchronize(p->st));
    if (outputs)
        for (int i = 0; i < NREG; i++) fe_to_bytes(outs[i], outputs + 16 * i);
    return ZK_OK;
}

int zk_vm_prove(zk_prover *p, zk_program *prog, const uint8_t *public_in, size_t num_public, const uint8_t *secret,
                size_t num_secret, uint32_t lwe_size, uint32_t delta, const uint8_t *last_row, const zk_options *opt,
                uint8_t *proof_out, size_t *proof_len, uint8_t *outputs, uint8_t *program_hash) {
    if (!p || !prog || !opt || !proof_len || (num_secret && !secret) || (num_public && !public_in))
        ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    ZK_REQUIRE_FULL_PROVER(p);
    const zk::vm::Inputs in{public_in, num_public, secret, num_secret, lwe_size, delta};
    fe outs[NREG], last[28];
    read_last(last_row, last);
    // ZK_VM_PREPROCESS=0: every column from the device trace (no per-program preprocessed columns)
    const char *pe = getenv("ZK_VM_PREPROCESS");
    const bool pre = !(pe && !strcmp(pe, "0")) && opt->blowup <= p->max_b && opt->blowup >= 8;
    size_t n = 0;
    zk_program::Fixed f{};
    uint32_t md = 0;
    FixedCols fx;
    struct ClearPrefix {  // a prefix not consumed by this call's proof must not reach another one
        zk_prover *p;
        ~ClearPrefix() { p->fix_prefix_blocks = 0; }
    } clear_prefix{p};
    if (pre) {
        // Processor::run + trace (vm/src/lib.rs:14-18): the program-only columns come from the program's preprocessed
        // coefficients / LDE; only the stack registers the program ever uses are generated
        ZK_TRY(fixed_columns(p, prog, in, opt->blowup, &f));
        fx.md = f.md;
        fx.fpolys = f.fpolys;
        fx.flde = f.flde;
        fx.lagr = f.lagr;
        fx.lagr_lde = f.lagr_lde;
        memcpy(fx.last, last, sizeof fx.last);
        // their share of the trace commitment needs only the last row: queued now, the GPU runs it while the host
        // runs the stack pass below (one call alone: the pass and this work no longer add up; 11.54-11.61 vs
        // 13.10-13.21 ms per call, profiles/r05k_vm_latency_ab_prefix.txt -- round 6 folded its switch into this default)
        if (prog->P.trace_len <= p->max_n) ZK_TRY(fixed_prefix(p, prog->P.trace_len, opt->blowup, fx));
        ZK_TRY(vm_generate(p, prog, in, last, GenMode{false, f.md}, &n, outs, &md));
        if ((int)md != f.md) ZK_FAIL(ZK_ERR_INVALID_ARG, "internal error: the stack depth depends on the inputs");
    } else {
        ZK_TRY(vm_generate(p, prog, in, last, GenMode{true, NREG}, &n, outs, nullptr));
    }
    // ExecutionProver::new(options, hash, output, server_key) + prove(trace) (:20-26) on the trace in HBM
    zk_pub_inputs pub;
    memset(&pub, 0, sizeof pub);
    fe_to_bytes(prog->P.hash[0], pub.program_hash[0]);
    fe_to_bytes(prog->P.hash[1], pub.program_hash[1]);
    for (int i = 0; i < NREG; i++) fe_to_bytes(outs[i], pub.stack_outputs[i]);
    pub.lwe_size = lwe_size;
    pub.delta = delta;
    if (outputs) memcpy(outputs, pub.stack_outputs, sizeof pub.stack_outputs);
    if (program_hash) memcpy(program_hash, pub.program_hash, sizeof pub.program_hash);
    if (!pre) return zk_prove_device(p, p->d_trace, n, opt, &pub, proof_out, proof_len, nullptr, nullptr);
    return prove_fixed(p, n, opt, &pub, &fx, proof_out, proof_len);
}

int zk_vm_prove_sharded(zk_comm *comm, zk_prover **provers, int nlocal, zk_program *prog, const uint8_t *public_in,
                        size_t num_public, const uint8_t *secret, size_t num_secret, uint32_t lwe_size, uint32_t delta,
                        const uint8_t *last_row, const zk_options *opt, uint8_t *proof_out, size_t *proof_len,
                        uint8_t *outputs, uint8_t *program_hash) {
    if (!comm || !provers || nlocal < 1 || !prog || !opt || !proof_len || (num_secret && !secret) ||
        (num_public && !public_in))
        ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    if (!last_row) ZK_FAIL(ZK_ERR_INVALID_ARG, "zk_vm_prove_sharded: last_row is required (every rank writes the same trace)");
    for (int l = 0; l < nlocal; l++)
        if (!provers[l]) ZK_FAIL(ZK_ERR_INVALID_ARG, "null prover");
    const zk::vm::Inputs in{public_in, num_public, secret, num_secret, lwe_size, delta};
    fe outs[NREG], last[28];
    read_last(last_row, last);
    size_t n = 0;
    const int G = comm->world;
    // ZK_VM_PREPROCESS=0: every column from the device trace, as zk_vm_prove
    const char *pe = getenv("ZK_VM_PREPROCESS");
    const bool pre = !(pe && !strcmp(pe, "0")) && opt->blowup == 8 && (G == 1 || G == 2 || G == 4 || G == 8);
    std::vector<FixedCols> fx(pre ? nlocal : 0);
    // Processor::run + trace on every local rank, each into its own trace buffer (the loopback communicator drives
    // several ranks from one process; one RCCL process holds one); with the preprocessed columns (built once per
    // program and rank, for the rank's own cosets) only the stack registers the program uses are generated
    for (int l = 0; l < nlocal; l++) {
        size_t nl = 0;
        if (pre) {
            zk_program::Fixed f{};
            const int bl = (int)opt->blowup / G;  // the rank's block of cosets
            ZK_TRY(fixed_columns(provers[l], prog, in, opt->blowup, &f, shard_rank_of(comm, l) * bl, bl));
            uint32_t md = 0;
            ZK_TRY(vm_generate(provers[l], prog, in, last, GenMode{false, f.md}, &nl, outs, &md));
            if ((int)md != f.md) ZK_FAIL(ZK_ERR_INVALID_ARG, "internal error: the stack depth depends on the inputs");
            fx[l].md = f.md;
            fx[l].fpolys = f.fpolys;
            fx[l].flde = f.flde;
            fx[l].lagr = f.lagr;
            fx[l].lagr_lde = f.lagr_lde;
            memcpy(fx[l].last, last, sizeof fx[l].last);
        } else {
            ZK_TRY(vm_generate(provers[l], prog, in, last, GenMode{true, NREG}, &nl, outs, nullptr));
        }
        n = nl;
    }
    zk_pub_inputs pub;
    memset(&pub, 0, sizeof pub);
    fe_to_bytes(prog->P.hash[0], pub.program_hash[0]);
    fe_to_bytes(prog->P.hash[1], pub.program_hash[1]);
    for (int i = 0; i < NREG; i++) fe_to_bytes(outs[i], pub.stack_outputs[i]);
    pub.lwe_size = lwe_size;
    pub.delta = delta;
    if (outputs) memcpy(outputs, pub.stack_outputs, sizeof pub.stack_outputs);
    if (program_hash) memcpy(program_hash, pub.program_hash, sizeof pub.program_hash);
    return prove_sharded_entry(comm, provers, nlocal, nullptr, n, opt, &pub, proof_out, proof_len, nullptr,
                               pre ? fx.data() : nullptr);
}

// diagnostics: the host stack pass's states every `stride` rows (CPU tests check them against host-written traces)
extern "C" int zk_diag_vm_states(const zk_program *prog, const uint8_t *public_in, size_t num_public,
                                 const uint8_t *secret, size_t num_secret, uint32_t lwe_size, uint32_t delta,
                                 size_t stride, size_t nstates, uint8_t *states_out, uint8_t *outputs) {
    if (!prog || !states_out || !stride) return ZK_ERR_INVALID_ARG;
    const zk::vm::Inputs in{public_in, num_public, secret, num_secret, lwe_size, delta};
    std::vector<VmState> st(nstates);
    fe outs[NREG];
    const int rc = zk::vm::stack_pass(prog->P, in, stride, nstates, st.data(), outs);
    if (rc) return rc;
    memcpy(states_out, st.data(), nstates * sizeof(VmState));
    if (outputs)
        for (int i = 0; i < NREG; i++) fe_to_bytes(outs[i], outputs + 16 * i);
    return ZK_OK;
}
