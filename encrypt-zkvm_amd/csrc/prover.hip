// prover.hip -- host orchestration of the gfx950 prove path and the C ABI (include/zkvm_gpu.h).
//
// zk_prove_device() runs winterfell 0.9's generate_proof stages for ProcessorAir
// (prover/src/lib.rs:40-77) on one GPU:
//   S0 coin seed                       host (Context::to_elements || PublicInputs::to_elements)
//   S2 trace iNTT + coset LDE + commit  ntt / hash_rows / merkle           (new_trace_lde)
//   S3 constraint evaluation           batch_inv + eval_constraints       (new_evaluator + evaluate)
//   S4 composition poly + commit       ntt(inverse) + comp_cross + ntt + hash_rows + merkle
//   S5 OOD frame, DEEP                 poly_eval + batch_inv + deep
//   S6 FRI layers + remainder          commit_fri_layer + fri_fold; remainder on host
//   S7 grinding + query positions      host
//   S8 openings                        gather kernels + host batch-proof assembly
//   S9 proof bytes                     host
// The public coin runs on the host and sees only 32-byte roots, so each commitment costs one
// small device->host copy.  Protocol choices are the ones of DESIGN.md "Protocol profile".
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "host_pool.hpp"
#include "prover_internal.hpp"
#include "rescue_consts.hpp"

namespace zk {
thread_local std::string g_err;
// ZK_HOST_TIMING=1: per proof, the host-only critical-path segments (the GPU idles during these) to stderr
struct HostTimer {
    bool on = getenv("ZK_HOST_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    std::string log;
    void start() { t = std::chrono::steady_clock::now(); }
    void stop(const char *what) {
        if (!on) return;
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count();
        char b[96];
        snprintf(b, sizeof b, " %s=%.1f", what, us);
        log += b;
    }
    ~HostTimer() {
        if (on && !log.empty()) fprintf(stderr, "[zk host us]%s\n", log.c_str());
    }
};
}
using namespace zk;

const char *zk_last_error(void) { return g_err.c_str(); }



struct zk_trace_lde {
    zk_prover *p;
    size_t n;
    uint32_t B;
    int width;
};

// ---------------------------------------------------------------- table construction
template <typename T>
static hipError_t upload(zk_prover *p, T **dst, const std::vector<T> &v) {
    hipError_t e = p->arena.alloc(dst, v.size());
    if (e != hipSuccess) return e;
    return hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
}
static std::vector<fe_ws> ws_of(const std::vector<fe> &v) {
    std::vector<fe_ws> w(v.size());
    for (size_t i = 0; i < v.size(); i++) w[i] = make_fe_ws(v[i]);
    return w;
}
static std::vector<fe_w2> w2_of(const std::vector<fe> &v) {
    std::vector<fe_w2> w(v.size());
    for (size_t i = 0; i < v.size(); i++) w[i] = make_fe_w2(v[i]);
    return w;
}

static hipError_t make_pow_table(zk_prover *p, fe s, size_t n, PowTable *out) {
    std::vector<fe> lo(2048), hi(n / 2048 + 1);
    lo[0] = fe_one();
    for (int t = 1; t < 2048; t++) lo[t] = fe_mul(lo[t - 1], s);
    fe s2048 = fe_mul(lo[2047], s);
    hi[0] = fe_one();
    for (size_t u = 1; u < hi.size(); u++) hi[u] = fe_mul(hi[u - 1], s2048);
    hipError_t e = upload(p, &out->lo, lo);
    if (e != hipSuccess) return e;
    return upload(p, &out->hi, hi);
}

static hipError_t make_ntt_tables(zk_prover *p, int log_n, NttTables *T) {
    T->log_n = log_n;
    // w_4096 powers, forward and inverse: built once per process (a function-local static is
    // initialised exactly once even when provers on several threads reach it together)
    struct Dft4096 {
        std::vector<fe> f, i;
        std::vector<fe_ws> fw, iw;
        std::vector<fe_w2> f2, i2;
        Dft4096() : f(2048), i(2048) {
            const fe w = h_root_of_unity(12), wi = h_inv(w);
            f[0] = i[0] = fe_one();
            for (int t = 1; t < 2048; t++) {
                f[t] = fe_mul(f[t - 1], w);
                i[t] = fe_mul(i[t - 1], wi);
            }
            fw = ws_of(f);
            iw = ws_of(i);
            f2 = w2_of(f);
            i2 = w2_of(i);
        }
    };
    static const Dft4096 d4096;
    hipError_t e = upload(p, &T->dft_fwd, d4096.f);
    if (e == hipSuccess) e = upload(p, &T->dft_inv, d4096.i);
    if (e == hipSuccess) e = upload(p, &T->dft_fwd_ws, d4096.fw);
    if (e == hipSuccess) e = upload(p, &T->dft_inv_ws, d4096.iw);
    if (e == hipSuccess) e = upload(p, &T->dft_fwd_w2, d4096.f2);
    if (e == hipSuccess) e = upload(p, &T->dft_inv_w2, d4096.i2);
    size_t n = (size_t)1 << log_n;
    fe w = h_root_of_unity(log_n);
    PowTable f, i;
    if (e == hipSuccess) e = make_pow_table(p, w, n, &f);
    if (e == hipSuccess) e = make_pow_table(p, h_inv(w), n, &i);
    T->fwd_lo = f.lo;
    T->fwd_hi = f.hi;
    T->inv_lo = i.lo;
    T->inv_hi = i.hi;
    return e;
}

// Periodic columns (air/src/lib.rs:201-225): CYCLE_MASK and the 8 ARK columns, interpolated over
// <w_16> and evaluated at (3 * w_CE^i)^(n/16) for the 128 distinct CE steps i mod 128.
static std::vector<fe> periodic_table(size_t n) {
    std::vector<std::vector<fe>> cols(9, std::vector<fe>(16));
    for (int r = 0; r < 16; r++) {
        cols[0][r] = fe_make(r < 14 ? 1 : 0);
        for (int c = 0; c < 8; c++) cols[1 + c][r] = fe_make(ZK_ARK[8 * r + c][0], ZK_ARK[8 * r + c][1]);
    }
    for (auto &c : cols) h_interp_coset(c, fe_one());
    const int log_ce = ilog2(8 * n);
    fe w = h_root_of_unity(log_ce), x = fe_make(3);
    std::vector<fe> out(128 * 9);
    for (int i = 0; i < 128; i++) {
        fe y = h_pow(x, n / 16);
        for (int j = 0; j < 9; j++) out[i * 9 + j] = h_poly_eval(cols[j].data(), 16, y);
        x = fe_mul(x, w);
    }
    return out;
}

int zk::get_plan(zk_prover *p, size_t n, uint32_t B, Plan **out) {
    auto key = std::make_pair(ilog2(n), ilog2(B));
    auto it = p->plans.find(key);
    if (it != p->plans.end()) {
        *out = it->second.get();
        return ZK_OK;
    }
    auto pl = std::make_unique<Plan>();
    pl->log_n = key.first;
    pl->log_b = key.second;
    ZK_CHECK_HIP(make_ntt_tables(p, pl->log_n, &pl->Tn));
    if (pl->log_n > 12) {  // four-step NTTs: inter-pass twiddle tables (2n elements)
        ZK_CHECK_HIP(p->arena.alloc(&pl->Tn.fwd_pass, n));
        ZK_CHECK_HIP(p->arena.alloc(&pl->Tn.inv_pass, n));
        ZK_CHECK_HIP(p->arena.alloc(&pl->Tn.inv_pass_n, n));
        pl->Tn.inv_n = h_inv(fe_make(n));
        make_pass_twiddles(p->st, pl->Tn);
    }
    ZK_CHECK_HIP(make_ntt_tables(p, pl->log_n + 3, &pl->Tce));
    ZK_CHECK_HIP(make_ntt_tables(p, pl->log_n + pl->log_b, &pl->TN));
    fe wN = h_root_of_unity(pl->log_n + pl->log_b), wce = h_root_of_unity(pl->log_n + 3);
    std::vector<fe> xrN(B), xrce(8), xnN(B);
    fe s = fe_make(3);
    // coset-LDE tables (CosetTables, B * n elements: 128 MiB at n = 2^20, B = 8)
    if (pl->log_n <= 12) {
        ZK_CHECK_HIP(p->arena.alloc(&pl->ct.full, (size_t)B * n));
    } else {
        ZK_CHECK_HIP(p->arena.alloc(&pl->ct.pass, (size_t)B * n));
        ZK_CHECK_HIP(p->arena.alloc(&pl->ct.stage, (size_t)B * 4096));
    }
    const int log_n2 = ntt_log_n2(pl->log_n);  // pass-1 line length of the four-step split (as in ntt_run())
    const size_t n2 = (size_t)1 << log_n2, n1 = n >> log_n2;
    std::vector<fe> stage(pl->log_n > 12 ? (size_t)B * 4096 : 0);
    for (uint32_t r = 0; r < B; r++) {
        xrN[r] = s;
        xnN[r] = h_pow(s, n);
        PowTable t;
        ZK_CHECK_HIP(make_pow_table(p, s, n, &t));
        if (pl->log_n <= 12) {
            pow_expand(p->st, t.lo, t.hi, n, pl->ct.full + (size_t)r * n);
        } else {
            // pass[r][k1 n2 + j2] = s^k1 w_n^(j2 k1); stage[r][h + j] = c^(n2/2h) w_2h^j with c = s^n1
            coset_pass_tables(p->st, t.lo, t.hi, pl->Tn.fwd_pass, pl->log_n, log_n2, pl->ct.pass + (size_t)r * n);
            const fe c = h_pow(s, n1);
            for (size_t h = 1; h < n2; h *= 2) {
                const fe w = h_root_of_unity(ilog2(2 * h));
                fe v = h_pow(c, n2 / (2 * h));
                for (size_t j = 0; j < h; j++) {
                    stage[(size_t)r * 4096 + h + j] = v;
                    v = fe_mul(v, w);
                }
            }
        }
        pl->coset.push_back(t);
        s = fe_mul(s, wN);
    }
    if (pl->log_n > 12) {
        ZK_CHECK_HIP(hipMemcpy(pl->ct.stage, stage.data(), stage.size() * sizeof(fe), hipMemcpyHostToDevice));
        ZK_CHECK_HIP(upload(p, &pl->ct.stage_ws, ws_of(stage)));
        ZK_CHECK_HIP(upload(p, &pl->ct.stage_w2, w2_of(stage)));
    }
    s = fe_make(3);
    for (int r = 0; r < 8; r++) {
        xrce[r] = s;
        s = fe_mul(s, wce);
    }
    ZK_CHECK_HIP(upload(p, &pl->xr_N, xrN));
    ZK_CHECK_HIP(upload(p, &pl->xn_N, xnN));
    ZK_CHECK_HIP(upload(p, &pl->xr_ce, xrce));
    ZK_CHECK_HIP(make_pow_table(p, h_inv(fe_make(3)), n, &pl->inv3));
    ZK_CHECK_HIP(upload(p, &pl->periodic, periodic_table(n)));
    if (pl->log_n > 12) {
        // e_(n-1)'s interpolant and coset LDE (the sparse trace columns': SparseCols).  A rank-sized prover holds the
        // LDE of its own cosets only (plan_rank_tables, once its rank is known)
        ZK_CHECK_HIP(p->arena.alloc(&pl->lagr, n));
        const bool full = p->shard_world <= 1;
        if (full) {
            ZK_CHECK_HIP(p->arena.alloc(&pl->lagr_lde, (size_t)B * n));
            pl->lde_cos = (int)B;
        }
        std::vector<fe> e(n, fe_zero());
        e[n - 1] = fe_one();
        fe *de = nullptr;
        ZK_CHECK_HIP(hipMalloc(&de, n * sizeof(fe)));
        hipError_t err = hipMemcpy(de, e.data(), n * sizeof(fe), hipMemcpyHostToDevice);
        if (err == hipSuccess) {
            const fe inv_n = h_inv(fe_make(n));
            ntt(p->st, pl->Tn, de, n, pl->lagr, n, 1, true, nullptr, &inv_n, p->tmp);
            if (full) ntt_lde(p->st, pl->Tn, pl->ct, pl->lagr, n, 1, 0, 1, (int)B, pl->lagr_lde, (size_t)B * n, n, p->tmp);
            err = hipStreamSynchronize(p->st);
        }
        (void)hipFree(de);
        ZK_CHECK_HIP(err);
    }
    ZK_CHECK_HIP(hipStreamSynchronize(p->st));
    *out = pl.get();
    p->plans[key] = std::move(pl);
    return ZK_OK;
}

Fe8 zk::ce_inv_zn(int log_n) {
    const size_t n = (size_t)1 << log_n;
    const fe wce = h_root_of_unity(log_n + 3);
    Fe8 z;
    fe x = fe_make(3);
    for (int r = 0; r < 8; r++, x = fe_mul(x, wce)) z.v[r] = h_inv(fe_sub(h_pow(x, n), fe_one()));
    return z;
}

const fe *zk::boundary_inverses(zk_prover *p, Plan *pl) {
    if (!pl->bnd_inv) {
        const size_t CE = (size_t)8 << pl->log_n, n = (size_t)1 << pl->log_n;
        if (p->arena.alloc(&pl->bnd_inv, 3 * CE) != hipSuccess) return nullptr;
        const fe g = h_root_of_unity(pl->log_n);
        divisor_tables(p->st, pl->Tn, pl->xr_ce, 3, pl->log_n, h_pow(g, n - 1), h_pow(g, n - 2), ce_inv_zn(pl->log_n),
                       pl->bnd_inv);
    }
    return pl->bnd_inv;
}

// ---------------------------------------------------------------- prover object
int zk_device_count(int *count) {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    if (count) *count = c;
    return ZK_OK;
}

// One upload stream per device for the process (created on first use, kept for the process's lifetime), shared by
// every prover on that device, with the mutex that keeps one prover's copy and its event record adjacent.
static int shared_upload_stream(int device, hipStream_t *st, std::mutex **mu, std::atomic<int> **busy) {
    struct Up {
        hipStream_t st = nullptr;
        std::mutex mu;
        std::atomic<int> busy{0};
    };
    static std::mutex reg_mu;
    static std::map<int, Up *> reg;  // process lifetime: never freed
    std::lock_guard<std::mutex> lk(reg_mu);
    Up *&u = reg[device];
    if (!u) {
        auto fresh = std::make_unique<Up>();
        ZK_CHECK_HIP(hipStreamCreateWithFlags(&fresh->st, hipStreamNonBlocking));
        u = fresh.release();
    }
    *st = u->st;
    *mu = &u->mu;
    *busy = &u->busy;
    return ZK_OK;
}

int zk::upload_gate(zk_prover *p, hipEvent_t ev) {
    (void)p;
    ZK_CHECK_HIP(hipEventSynchronize(ev));
    return ZK_OK;
}

void zk::upload_drain(zk_prover *p) {
    for (auto &e : p->ev_up)
        if (e) (void)hipEventSynchronize(e);
}

// world = 0: a full prover; world = G: one rank of a G-way coset-sharded proof (blowup 8), whose LDE-domain
// buffers (trace / composition LDE, DEEP, NTT scratch, Merkle subtrees) hold N / G points instead of N
static int create_prover(int device, size_t max_n, uint32_t max_b, int world, zk_prover **out) {
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess || cnt == 0) ZK_FAIL(ZK_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= cnt) ZK_FAIL(ZK_ERR_INVALID_ARG, "device index out of range");
    ZK_CHECK_HIP(hipSetDevice(device));
    // The host waits on the prover stream a few times per proof (transcript round trips): spin instead
    // of yielding (A/B: -0.05 ms per 2^20 proof).  PROCESS-WIDE side effect (documented at zk_prover_create
    // in zkvm_gpu.h): hipDeviceScheduleSpin applies to every stream sync of the process on this device, so
    // each waiting host thread busy-spins.  Only takes effect if this is the first use of the device in the
    // process; ZK_SPIN_WAIT=0 keeps the runtime's default (yield).
    {
        const char *e = getenv("ZK_SPIN_WAIT");
        if (!e || atoi(e)) {
            (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
            (void)hipGetLastError();  // refused once the context exists: leave no sticky error behind
        }
    }
    auto p = std::make_unique<zk_prover>();
    p->device = device;
    p->max_n = max_n;
    p->max_b = max_b;
    ZK_CHECK_HIP(hipStreamCreateWithFlags(&p->st, hipStreamNonBlocking));
    ZK_TRY(shared_upload_stream(device, &p->up, &p->up_mu, &p->dev_busy));
    for (auto &e : p->ev_up) ZK_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ZK_CHECK_HIP(upload_rescue_consts(p->st));
    const size_t n = max_n, N = max_n * max_b, CE = 8 * max_n;
    // Nl: LDE-domain points this prover holds (all N, or the N / G of one sharded rank)
    if (world == 1) world = 0;  // one rank holds the whole domain: a full prover
    p->shard_world = world;
    const size_t Nl = world ? N / (size_t)world : N;
    DeviceArena &A = p->arena;
    ZK_CHECK_HIP(A.alloc(&p->d_trace, (size_t)W * n));
    // trace polynomials; as a rank of a sharded proof, G slices of ceil(W / G) columns (the in-place all-gather of
    // shard.hip): 8 ceil(W / 8) columns cover G = 1, 2, 4, 8
    ZK_CHECK_HIP(A.alloc(&p->polys, (size_t)8 * ((W + 7) / 8) * n));
    // NTT scratch: the four-step intermediate of a whole 8-coset LDE of the trace (28 x 8 x n; a sharded rank's
    // cosets: 28 x 8/G x n, at least the 28 x n of the interpolation)
    ZK_CHECK_HIP(A.alloc(&p->tmp, (size_t)W * (world ? std::max<size_t>(n, Nl) : 8 * n)));
    ZK_CHECK_HIP(A.alloc(&p->lde, (size_t)W * Nl));
    ZK_CHECK_HIP(A.alloc(&p->comp, CE));
    ZK_CHECK_HIP(A.alloc(&p->ctmp, CE));
    ZK_CHECK_HIP(A.alloc(&p->cpolys, (size_t)ZK_MAX_CCOLS * n));
    ZK_CHECK_HIP(A.alloc(&p->clde, (size_t)8 * Nl));
    ZK_CHECK_HIP(A.alloc(&p->deep, Nl));
    if (!world) ZK_CHECK_HIP(A.alloc(&p->ulde, N));  // the single path's DEEP LDE
    ZK_CHECK_HIP(A.alloc(&p->dscratch, 4 * (2048 + n / 2048 + 2) + 3 * n + 2 * (n / 256 + 1)));
    // FRI layers: sum over layers of L/fold values and 2*L/fold digests; worst case fold = 2
    ZK_CHECK_HIP(A.alloc(&p->fri, N + 16));
    ZK_CHECK_HIP(A.alloc(&p->leaves, 32 * Nl));
    ZK_CHECK_HIP(A.alloc(&p->nodes, 32 * Nl));
    ZK_CHECK_HIP(A.alloc(&p->cleaves, 32 * Nl));
    ZK_CHECK_HIP(A.alloc(&p->cnodes, 32 * Nl));
    // digest scratch: a sharded rank's all-to-all send + receive areas (64 B per local point), and the digests of
    // the FRI layers >= 1 (at most 32 B per point of the whole domain, fold 2)
    ZK_CHECK_HIP(A.alloc(&p->fri_dig, (world ? std::max<size_t>(64 * Nl, 32 * N) : 64 * N) + 64));
    ZK_CHECK_HIP(A.alloc(&p->partials, (size_t)(2 * ZK_MAX_COLS + ZK_MAX_CCOLS) * ood_waves(max_n)));
    ZK_CHECK_HIP(A.alloc(&p->ood_tab, (size_t)128 + 2 * ood_waves(max_n)));
    ZK_CHECK_HIP(A.alloc(&p->ood, 256));
    ZK_CHECK_HIP(A.alloc(&p->gather_out, ZK_GATHER_CAP));
    ZK_CHECK_HIP(A.alloc(&p->gather_idx, ZK_GATHER_CAP));
    // the largest read is the last FRI layer: up to ZK_MAX_REMAINDER * blowup values, two planes over E
    p->io_cap = ((size_t)64 << 10) + (size_t)2 * ZK_MAX_REMAINDER * p->max_b * sizeof(fe);
    ZK_CHECK_HIP(hipHostMalloc((void **)&p->h_io, p->io_cap, hipHostMallocDefault));
    p->io_pending.reserve(64);
    ZK_CHECK_HIP(hipHostMalloc((void **)&p->h_gather_idx, ZK_GATHER_CAP * sizeof(uint64_t), hipHostMallocDefault));
    ZK_CHECK_HIP(hipHostMalloc((void **)&p->h_gather_out, ZK_GATHER_CAP * sizeof(fe), hipHostMallocDefault));
    ZK_CHECK_HIP(A.alloc(&p->flag, 4));
    ZK_CHECK_HIP(A.alloc((uint8_t **)&p->air_consts, sizeof(AirConsts)));
    ZK_CHECK_HIP(A.alloc((uint8_t **)&p->deep_consts, sizeof(DeepConsts)));
    ZK_CHECK_HIP(A.alloc((uint8_t **)&p->fold_consts, sizeof(FoldConsts)));
    ZK_CHECK_HIP(A.alloc(&p->fri_seed, 32));
    ZK_CHECK_HIP(A.alloc(&p->fri_alphas, 2 * ZK_MAX_FRI_LAYERS));
    *out = p.release();
    return ZK_OK;
}

int zk_prover_create(int device, size_t max_n, uint32_t max_b, zk_prover **out) {
    if (!out || max_n < 16 || (max_n & (max_n - 1)) || max_b < 8 || (max_b & (max_b - 1)) || max_b > 64)
        ZK_FAIL(ZK_ERR_INVALID_ARG, "zk_prover_create: max_trace_len must be a power of two >= 16, blowup in [8, 64]");
    return create_prover(device, max_n, max_b, 0, out);
}

int zk_prover_create_shard(int device, size_t max_n, int world, zk_prover **out) {
    if (!out || max_n < 16 || (max_n & (max_n - 1)) || (world != 1 && world != 2 && world != 4 && world != 8))
        ZK_FAIL(ZK_ERR_INVALID_ARG, "zk_prover_create_shard: max_trace_len a power of two >= 16, world 1, 2, 4 or 8");
    return create_prover(device, max_n, 8, world, out);
}

void zk_prover_destroy(zk_prover *p) {
    if (!p) return;
    (void)hipSetDevice(p->device);
    (void)hipStreamSynchronize(p->st);
    upload_drain(p);
    for (auto &e : p->stage_pool) (void)hipEventDestroy(e);
    for (auto &e : p->xchg_pool) (void)hipEventDestroy(e);
    if (p->cst) {
        (void)hipStreamSynchronize(p->cst);
        (void)hipStreamDestroy(p->cst);
    }
    if (p->ev_ready) (void)hipEventDestroy(p->ev_ready);
    for (auto &e : p->ev_up)
        if (e) (void)hipEventDestroy(e);
    if (p->ev_vm) (void)hipEventDestroy(p->ev_vm);
    (void)hipStreamDestroy(p->st);
    if (p->h_io) (void)hipHostFree(p->h_io);
    if (p->h_gather_idx) (void)hipHostFree(p->h_gather_idx);
    if (p->h_gather_out) (void)hipHostFree(p->h_gather_out);
    if (p->h_vm) (void)hipHostFree(p->h_vm);
    if (p->sp_h) (void)hipHostFree(p->sp_h);
    if (p->h_pack) (void)hipHostFree(p->h_pack);
    delete p->open;
    delete p;
}

// ---------------------------------------------------------------- process-wide prover pool
// The reference builds its prover per call (ExecutionProver::new in vm::prove, vm/src/lib.rs:24).  A zk_prover is
// ~12.5 GB of HBM at 2^20 plus per-size tables built by its first proof, so the drop-in keeps released provers for
// the next acquire on the same device instead (zk_prover_acquire / zk_prover_release).
namespace {
struct Pool {
    std::mutex mu;
    std::vector<zk_prover *> idle;
};
Pool &pool() {
    static Pool *P = new Pool();  // process lifetime (provers released at exit are reclaimed with the process)
    return *P;
}
}  // namespace

int zk_prover_acquire(int device, size_t max_n, uint32_t max_b, zk_prover **out) {
    if (!out) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    {
        Pool &P = pool();
        std::lock_guard<std::mutex> lk(P.mu);
        // the smallest idle full prover of this device that fits
        size_t best = P.idle.size();
        for (size_t i = 0; i < P.idle.size(); i++) {
            const zk_prover *q = P.idle[i];
            if (q->device != device || q->shard_world || q->max_n < max_n || q->max_b < max_b) continue;
            if (best == P.idle.size() || q->max_n * q->max_b < P.idle[best]->max_n * P.idle[best]->max_b) best = i;
        }
        if (best < P.idle.size()) {
            *out = P.idle[best];
            P.idle.erase(P.idle.begin() + (long)best);
            return ZK_OK;
        }
    }
    return zk_prover_create(device, max_n, max_b, out);
}

void zk_prover_release(zk_prover *p) {
    if (!p) return;
    if (p->shard_world) {  // rank-sized provers are not pooled
        zk_prover_destroy(p);
        return;
    }
    (void)hipSetDevice(p->device);
    (void)hipStreamSynchronize(p->st);
    Pool &P = pool();
    std::lock_guard<std::mutex> lk(P.mu);
    P.idle.push_back(p);
}

int zk_prover_pool_trim(int device) {
    std::vector<zk_prover *> drop;
    {
        Pool &P = pool();
        std::lock_guard<std::mutex> lk(P.mu);
        for (size_t i = 0; i < P.idle.size();)
            if (device < 0 || P.idle[i]->device == device) {
                drop.push_back(P.idle[i]);
                P.idle.erase(P.idle.begin() + (long)i);
            } else {
                i++;
            }
    }
    for (zk_prover *p : drop) zk_prover_destroy(p);
    return (int)drop.size();
}

int zk_prover_trace_buffer(zk_prover *p, void **d_trace) {
    if (!p || !d_trace) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    *d_trace = p->d_trace;
    return ZK_OK;
}

// ---------------------------------------------------------------- stage timing
void zk::stage_begin(zk_prover *p) {
    p->stage_names.clear();
    p->stage_done = false;
    p->xchg.clear();
    p->xchg_next = 0;
    p->sched.clear();
}
void zk::stage_mark(zk_prover *p, const char *name) {
    const size_t i = p->stage_names.size();
    if (i == p->stage_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;  // timing only: a missing mark is not an error
        p->stage_pool.push_back(e);
    }
    (void)hipEventRecord(p->stage_pool[i], p->st);
    p->stage_names.push_back(name);
}
// the proof is complete (its stream synchronized): its stage events may be read until the next proof
void zk::stage_collect(zk_prover *p) { p->stage_done = true; }

int zk_prover_stage_times(zk_prover *p, const char **names, float *ms, int cap, int *count) {
    if (!p) ZK_FAIL(ZK_ERR_INVALID_ARG, "null prover");
    p->stage_ms.clear();
    if (p->stage_done)
        for (size_t i = 1; i < p->stage_names.size(); i++) {
            float t = 0;
            (void)hipEventElapsedTime(&t, p->stage_pool[i - 1], p->stage_pool[i]);
            p->stage_ms.push_back({p->stage_names[i], t});
        }
    int k = (int)p->stage_ms.size();
    for (int i = 0; i < k && i < cap; i++) {
        if (names) names[i] = p->stage_ms[i].first;
        if (ms) ms[i] = p->stage_ms[i].second;
    }
    if (count) *count = k;
    return ZK_OK;
}

int zk_prover_proof_info(const zk_prover *p, zk_proof_info *out) {
    if (!p || !out) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    memset(out, 0, sizeof *out);
    out->schedule = p->last_sched;
    out->hint_redos = p->hint_redos;
    for (const auto &h : p->hint_sets) out->hint_sets += h.n != 0 && h.have ? 1u : 0u;
    out->hinted_sparse = p->sp_hinted;
    out->derived = p->clk_used ? 1u : 0u;
    return ZK_OK;
}

int zk_prover_upload_stats(zk_prover *p, uint64_t *bytes, uint32_t *sparse_cols, uint32_t *narrow8_cols,
                           uint32_t *narrow32_cols) {
    if (!p) ZK_FAIL(ZK_ERR_INVALID_ARG, "null prover");
    if (bytes) *bytes = p->up_bytes;
    if (sparse_cols) *sparse_cols = p->up_sparse;
    if (narrow8_cols) *narrow8_cols = p->up_nw8;
    if (narrow32_cols) *narrow32_cols = p->up_nw32;
    return ZK_OK;
}

int zk_prover_upload_derived(zk_prover *p, uint32_t *derived_cols) {
    if (!p || !derived_cols) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    *derived_cols = p->clk_used ? 1u : 0u;
    return ZK_OK;
}

int zk_prover_exchange_stats_ex(zk_prover *p, const char **names, float *ms, float *exposed_ms, double *bytes,
                                int *calls, int cap, int *count) {
    if (!p) ZK_FAIL(ZK_ERR_INVALID_ARG, "null prover");
    std::vector<const char *> nm;
    std::vector<float> t, w;
    std::vector<double> b;
    std::vector<int> c;
    if (p->stage_done)
        for (const auto &r : p->xchg) {
            float x = 0, y = 0;
            (void)hipEventElapsedTime(&x, p->xchg_pool[r.ev], p->xchg_pool[r.ev + 1]);
            if (r.waited) (void)hipEventElapsedTime(&y, p->xchg_pool[r.ev + 2], p->xchg_pool[r.ev + 3]);
            size_t i = 0;
            while (i < nm.size() && strcmp(nm[i], r.name)) i++;
            if (i == nm.size()) {
                nm.push_back(r.name);
                t.push_back(0);
                w.push_back(0);
                b.push_back(0);
                c.push_back(0);
            }
            t[i] += x;
            w[i] += y;
            b[i] += r.bytes;
            c[i] += 1;
        }
    const int k = (int)nm.size();
    for (int i = 0; i < k && i < cap; i++) {
        if (names) names[i] = nm[i];
        if (ms) ms[i] = t[i];
        if (exposed_ms) exposed_ms[i] = w[i];
        if (bytes) bytes[i] = b[i];
        if (calls) calls[i] = c[i];
    }
    if (count) *count = k;
    return ZK_OK;
}

int zk_prover_exchange_stats(zk_prover *p, const char **names, float *ms, double *bytes, int *calls, int cap,
                             int *count) {
    return zk_prover_exchange_stats_ex(p, names, ms, nullptr, bytes, calls, cap, count);
}

int zk_prover_shard_schedule(zk_prover *p, char *buf, size_t cap, size_t *len) {
    if (!p || !len) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    std::string js = "{\"world\": " + std::to_string(p->sched_world) +
                     ", \"measure\": " + (p->sched_measure ? "true" : "false") + ", \"entries\": [";
    char tmp[256];
    auto el = [&](size_t a, size_t b) {
        float x = 0;
        (void)hipEventElapsedTime(&x, p->xchg_pool[a], p->xchg_pool[b]);
        return x;
    };
    if (p->stage_done)
        for (size_t i = 0; i < p->sched.size(); i++) {
            const auto &e = p->sched[i];
            // the compute segment before this entry
            const float seg = i ? el(p->sched[i - 1].post, e.pre) : 0.f;
            snprintf(tmp, sizeof tmp, "%s{\"seg_ms\": %.5f, \"lead\": %s}", i ? ", " : "", seg,
                     e.lead ? "true" : "false");
            js += tmp;
            if (e.kind == 'S' || e.kind == 'W') {
                const auto &r = p->xchg[e.x];
                if (e.kind == 'S')
                    snprintf(tmp, sizeof tmp, ", {\"start\": %d, \"name\": \"%s\", \"op\": \"%s\", \"bytes\": %.0f, "
                             "\"ms\": %.5f}", e.x, r.name, r.op ? "ag" : "a2a", r.bytes, el(r.ev, r.ev + 1));
                else
                    snprintf(tmp, sizeof tmp, ", {\"wait\": %d, \"exposed_ms\": %.5f}", e.x, el(e.pre, e.post));
                js += tmp;
            }
        }
    js += "]}";
    *len = js.size() + 1;
    if (!buf || cap < js.size() + 1) ZK_FAIL(ZK_ERR_BUFFER_TOO_SMALL, "schedule buffer too small");
    memcpy(buf, js.c_str(), js.size() + 1);
    return ZK_OK;
}

int zk_prover_set_upload_schedule(zk_prover *p, int schedule) {
    if (!p) ZK_FAIL(ZK_ERR_INVALID_ARG, "null prover");
    if (schedule < ZK_SCHED_AUTO || schedule > ZK_SCHED_LATENCY) ZK_FAIL(ZK_ERR_INVALID_ARG, "unknown upload schedule");
    p->upload_sched = schedule;
    return ZK_OK;
}

int zk_prover_profile(zk_prover *p, int enable) {
    if (!p) ZK_FAIL(ZK_ERR_INVALID_ARG, "null prover");
    profiler().on = enable != 0;
    profiler().reset();
    return ZK_OK;
}

void zk::collect_kernel_stats(zk_prover *p) {
    KernelProfiler &P = profiler();
    if (!P.on) return;
    (void)hipStreamSynchronize(p->st);
    for (auto &r : P.recs) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, r.a, r.b);
        size_t i = 0;
        for (; i < p->kstat_names.size(); i++)
            if (p->kstat_names[i] == r.name) break;
        if (i == p->kstat_names.size()) {
            p->kstat_names.push_back(r.name);
            p->kstat_ms.push_back(0);
            p->kstat_n.push_back(0);
            p->kstat_bytes.push_back(0);
            p->kstat_muls.push_back(0);
            p->kstat_addsubs.push_back(0);
        }
        p->kstat_ms[i] += ms;
        p->kstat_n[i] += 1;
        p->kstat_bytes[i] += r.bytes;
        p->kstat_muls[i] += r.muls;
        p->kstat_addsubs[i] += r.addsubs;
    }
    P.reset();
}

int zk_prover_kernel_stats(zk_prover *p, const char **names, float *total_ms, int *launches, double *total_bytes,
                           int cap, int *count) {
    if (!p) ZK_FAIL(ZK_ERR_INVALID_ARG, "null prover");
    int k = (int)p->kstat_names.size();
    for (int i = 0; i < k && i < cap; i++) {
        if (names) names[i] = p->kstat_names[i].c_str();
        if (total_ms) total_ms[i] = p->kstat_ms[i];
        if (launches) launches[i] = p->kstat_n[i];
        if (total_bytes) total_bytes[i] = p->kstat_bytes[i];
    }
    if (count) *count = k;
    if (!names && !total_ms && !launches && !total_bytes) {  // reset request
        p->kstat_names.clear();
        p->kstat_ms.clear();
        p->kstat_n.clear();
        p->kstat_bytes.clear();
        p->kstat_muls.clear();
        p->kstat_addsubs.clear();
    }
    return ZK_OK;
}

int zk_prover_kernel_ops(zk_prover *p, double *total_muls, double *total_addsubs, int cap, int *count) {
    if (!p) ZK_FAIL(ZK_ERR_INVALID_ARG, "null prover");
    const int k = (int)p->kstat_names.size();
    for (int i = 0; i < k && i < cap; i++) {
        if (total_muls) total_muls[i] = p->kstat_muls[i];
        if (total_addsubs) total_addsubs[i] = p->kstat_addsubs[i];
    }
    if (count) *count = k;
    return ZK_OK;
}

// ---------------------------------------------------------------- Merkle batch openings
void zk::plan_batch(size_t nl, const std::vector<uint64_t> &idx, BatchPlan &bp) {
    int depth = ilog2(nl);
    bp.norm.clear();
    for (uint64_t i : idx) bp.norm.push_back(i & ~1ULL);
    std::sort(bp.norm.begin(), bp.norm.end());
    bp.norm.erase(std::unique(bp.norm.begin(), bp.norm.end()), bp.norm.end());
    bp.paths.resize(bp.norm.size());
    for (auto &path : bp.paths) path.clear();  // keep their capacity across proofs
    std::vector<uint64_t> &next = bp.next, &cur = bp.cur;
    next.clear();
    for (size_t i = 0; i < bp.norm.size(); i++) {
        for (uint64_t l = bp.norm[i]; l < bp.norm[i] + 2; l++)
            if (std::find(idx.begin(), idx.end(), l) == idx.end()) bp.paths[i].push_back({0, l});
        next.push_back((bp.norm[i] + nl) >> 1);
    }
    for (int lvl = 1; lvl < depth; lvl++) {
        std::swap(cur, next);
        next.clear();
        for (size_t i = 0; i < cur.size(); i++) {
            uint64_t sib = cur[i] ^ 1;
            if (i + 1 < cur.size() && cur[i + 1] == sib)
                i++;
            else
                bp.paths[i].push_back({1, sib});
            next.push_back(sib >> 1);
        }
    }
}

BatchPlan zk::plan_batch(size_t nl, const std::vector<uint64_t> &idx) {
    BatchPlan bp;
    plan_batch(nl, idx, bp);
    return bp;
}

// ---------------------------------------------------------------- the prove path
// ---------------------------------------------------------------- protocol steps (host side)
int zk::check_prove_args(size_t n, size_t max_n, uint32_t max_b, const zk_options *o, const zk_pub_inputs *pub) {
    if (!o || !pub) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    if ((o->field_extension != 1 && o->field_extension != 2) || o->blowup < 8 || (o->blowup & (o->blowup - 1)) ||
        (o->fri_folding != 2 && o->fri_folding != 4 && o->fri_folding != 8 && o->fri_folding != 16) ||
        ((o->fri_rem_max_deg + 1) & o->fri_rem_max_deg) || o->fri_rem_max_deg + 1 > ZK_MAX_REMAINDER ||
        o->num_queries == 0 || o->num_queries > ZK_MAX_QUERIES)
        ZK_FAIL(ZK_ERR_INVALID_ARG, "unsupported proof options");
    // winter-air ProofOptions::new asserts grinding_factor <= 32 (and the proof stores it as one byte)
    if (o->grinding > 32) ZK_FAIL(ZK_ERR_INVALID_ARG, "grinding factor must be at most 32");
    if (n < 16 || (n & (n - 1)) || n > max_n) ZK_FAIL(ZK_ERR_INVALID_ARG, "trace length must be a power of two in [16, max_trace_len]");
    if (o->blowup > max_b) ZK_FAIL(ZK_ERR_INVALID_ARG, "blowup exceeds the prover's max_blowup");
    if (pub->lwe_size == 0 || pub->lwe_size > 5)
        ZK_FAIL(ZK_ERR_INVALID_ARG, "lwe_size must be in [1, 5] (enforce_add2 reads 2*lwe_size stack items, constrains.rs:129)");
    if (o->num_queries >= n * o->blowup) ZK_FAIL(ZK_ERR_INVALID_ARG, "num_queries must be smaller than the LDE domain");
    return ZK_OK;
}

Coin zk::seed_coin(size_t n, const zk_options *opt, const zk_pub_inputs *pub) {
    std::vector<fe> e;
    e.push_back(fe_make((uint64_t)W << 16));
    e.push_back(fe_make(n));
    e.push_back(fe_make(ZK_P_LO));
    e.push_back(fe_make(ZK_P_HI));
    e.push_back(fe_make(((uint64_t)opt->field_extension << 16) | ((uint64_t)opt->fri_folding << 8) | opt->fri_rem_max_deg));
    e.push_back(fe_make(opt->grinding));
    e.push_back(fe_make(opt->blowup));
    e.push_back(fe_make(opt->num_queries));
    for (int i = 0; i < 2; i++) e.push_back(fe_from_bytes(pub->program_hash[i]));
    for (int i = 0; i < 16; i++) e.push_back(fe_from_bytes(pub->stack_outputs[i]));
    Coin coin;
    coin.init(e);
    return coin;
}

// assertions (air/src/lib.rs:170-195) sorted by (stride, first_step, column) [P3]; CE-coset constants
static void set_bnd1(AirConsts &K) {
    K.bnd1 = fe_zero();
    for (int k = 12; k < NUM_ASSERTS; k++) K.bnd1 = fe_add(K.bnd1, fe_mul(K.coeff_b[k], K.assert_val[k]));
}

static void air_static_consts(const zk_pub_inputs *pub, size_t n, AirConsts &K) {
    const int log_n = ilog2(n);
    const int first_cols[12] = {0, 7, 8, 11, 12, 13, 14, 15, 16, 17, 18, 19};
    int k = 0;
    for (int i = 0; i < 12; i++, k++) {
        K.assert_col[k] = first_cols[i];
        K.assert_grp[k] = 0;
        K.assert_val[k] = fe_zero();
    }
    for (int i = 0; i < 2; i++, k++) {
        K.assert_col[k] = 7 + i;
        K.assert_grp[k] = 1;
        K.assert_val[k] = fe_from_bytes(pub->program_hash[i]);
    }
    for (int i = 0; i < 8; i++, k++) {
        K.assert_col[k] = 12 + i;
        K.assert_grp[k] = 1;
        K.assert_val[k] = fe_from_bytes(pub->stack_outputs[i]);
    }
    // the divisor constants depend only on n: computed once per n and thread (8 inversions and
    // 10 exponentiations, host time the GPU would otherwise wait for on every proof)
    struct DivConsts {
        fe xr[8], inv_zn[8], g_last2, g_last1;
    };
    static thread_local std::map<size_t, DivConsts> cache;
    auto it = cache.find(n);
    if (it == cache.end()) {
        DivConsts d;
        const fe g = h_root_of_unity(log_n);
        fe wce = h_root_of_unity(log_n + 3), x = fe_make(3);
        for (int r = 0; r < 8; r++) {
            d.xr[r] = x;
            d.inv_zn[r] = h_inv(fe_sub(h_pow(x, n), fe_one()));  // x^n constant on CE coset r
            x = fe_mul(x, wce);
        }
        d.g_last2 = h_pow(g, n - 2);
        d.g_last1 = h_pow(g, n - 1);
        it = cache.emplace(n, d).first;
    }
    memcpy(K.xr, it->second.xr, sizeof K.xr);
    memcpy(K.inv_zn, it->second.inv_zn, sizeof K.inv_zn);
    K.g_last2 = it->second.g_last2;
    K.g_last1 = it->second.g_last1;
    K.delta = fe_make(pub->delta);
    K.lwe_size = (int)pub->lwe_size;
    set_bnd1(K);
}

void zk::draw_air_consts(Coin &coin, const zk_pub_inputs *pub, size_t n, AirConsts &K, zk_record &R) {
    memset(&K, 0, sizeof K);
    for (int k = 0; k < NUM_TCONS; k++) fe_to_bytes(K.coeff_t[k] = coin.draw(), R.coeff_t[k]);
    for (int k = 0; k < NUM_ASSERTS; k++) fe_to_bytes(K.coeff_b[k] = coin.draw(), R.coeff_b[k]);
    air_static_consts(pub, n, K);
}

void zk::draw_air_consts_ext(Coin &coin, const zk_pub_inputs *pub, size_t n, AirConsts &Ka, AirConsts &Kb,
                             zk_record &R) {
    memset(&Ka, 0, sizeof Ka);
    for (int k = 0; k < NUM_TCONS; k++) {
        const fe2 v = coin.draw_ext(2);
        Ka.coeff_t[k] = v.a;
        Kb.coeff_t[k] = v.b;
        fe_to_bytes(v.a, R.coeff_t[k]);
    }
    for (int k = 0; k < NUM_ASSERTS; k++) {
        const fe2 v = coin.draw_ext(2);
        Ka.coeff_b[k] = v.a;
        Kb.coeff_b[k] = v.b;
        fe_to_bytes(v.a, R.coeff_b[k]);
    }
    air_static_consts(pub, n, Ka);
    const AirConsts tmp = Kb;
    Kb = Ka;
    memcpy(Kb.coeff_t, tmp.coeff_t, sizeof Kb.coeff_t);
    memcpy(Kb.coeff_b, tmp.coeff_b, sizeof Kb.coeff_b);
    set_bnd1(Kb);
}

void zk::ood_reseed(Coin &coin, const fe *h, int C, zk_record &R) {
    for (int c = 0; c < W; c++) {
        fe_to_bytes(h[c], R.ood_trace_z[c]);
        fe_to_bytes(h[W + c], R.ood_trace_zg[c]);
    }
    for (int j = 0; j < C; j++) fe_to_bytes(h[2 * W + j], R.ood_constraints[j]);
    uint8_t d[32];
    hash_elems(h, 2 * W, d);  // T(z) || T(zg)
    coin.reseed(d);
    hash_elems(h + 2 * W, C, d);
    coin.reseed(d);
}

DeepConsts zk::draw_deep_consts(Coin &coin, const fe *h, int C, fe z, fe zg, zk_record &R) {
    DeepConsts D;
    memset(&D, 0, sizeof D);
    for (int c = 0; c < W; c++) fe_to_bytes(D.alpha_t[c] = coin.draw(), R.deep_t[c]);
    for (int j = 0; j < C; j++) fe_to_bytes(D.alpha_c[j] = coin.draw(), R.deep_c[j]);
    fe k1 = fe_zero(), k2 = fe_zero();
    for (int c = 0; c < W; c++) {
        k1 = fe_add(k1, fe_mul(D.alpha_t[c], h[c]));
        k2 = fe_add(k2, fe_mul(D.alpha_t[c], h[W + c]));
    }
    for (int j = 0; j < C; j++) k1 = fe_add(k1, fe_mul(D.alpha_c[j], h[2 * W + j]));
    D.k1 = k1;
    D.k2 = k2;
    D.z = z;
    D.zg = zg;
    return D;
}

int zk::fri_num_layers(size_t N, const zk_options *opt) {
    const size_t max_rem = (size_t)(opt->fri_rem_max_deg + 1) * opt->blowup;
    int nl = 0;
    for (size_t s = N; s > max_rem; s /= opt->fri_folding) nl++;
    return nl;
}

FoldConsts zk::fold_consts(fe alpha, uint32_t fold) {
    FoldConsts F;
    memset(&F, 0, sizeof F);
    const fe zeta_inv = h_inv(h_root_of_unity(ilog2(fold)));
    F.zinv[0] = fe_one();
    for (uint32_t t = 1; t < 16; t++) F.zinv[t] = t < fold ? fe_mul(F.zinv[t - 1], zeta_inv) : fe_zero();
    F.alpha = alpha;
    F.inv_offset = h_inv(fe_make(3));
    F.inv_fold = h_inv(fe_make(fold));
    return F;
}

int zk::remainder_step(std::vector<fe> &rv, uint32_t B, Coin &coin, zk_record &R, unsigned &degree_flag) {
    const size_t L = rv.size();
    h_interp_coset3_cached(rv);
    const size_t rl = L / B;
    for (size_t k = rl; k < L; k++)
        if (!fe_is_zero(rv[k])) degree_flag = 1;
    if (rl > ZK_MAX_REMAINDER) ZK_FAIL(ZK_ERR_INVALID_ARG, "remainder too large");
    R.remainder_len = (uint32_t)rl;
    for (size_t k = 0; k < rl; k++) fe_to_bytes(rv[k], R.remainder[k]);
    hash_elems(rv.data(), rl, R.remainder_commitment);
    coin.reseed(R.remainder_commitment);
    return ZK_OK;
}

// ---- FieldExtension::Quadratic host steps (shared by the single-GPU and sharded paths)
// hv = ood_eval_ext output (2 planes of np = 2W + C*2 values): E values of T(z), T(zg) and of the 2C base
// composition columns at z.  Builds the E frame e = T(z) ++ T(zg) ++ H(z) (H_c = P_c0 + X P_c1), its
// flattened form h (the serialization order), records the a components, reseeds the coin [P7, P15].
void zk::ood_reseed_ext(Coin &coin, const std::vector<fe> &hv, int C, zk_record &R, std::vector<fe2> &e,
                        std::vector<fe> &h) {
    const int np = 2 * W + 2 * C;
    e.assign(2 * W + C, fe2_zero());
    for (int c = 0; c < 2 * W; c++) e[c] = fe2{hv[c], hv[np + c]};
    for (int c = 0; c < C; c++) {
        const int s0 = 2 * W + 2 * c;
        e[2 * W + c] = fe2_add(fe2{hv[s0], hv[np + s0]}, fe2_mulX(fe2{hv[s0 + 1], hv[np + s0 + 1]}));
    }
    h.assign(2 * e.size(), fe_zero());
    for (size_t i = 0; i < e.size(); i++) {
        h[2 * i] = e[i].a;
        h[2 * i + 1] = e[i].b;
    }
    for (int c = 0; c < W; c++) {
        fe_to_bytes(e[c].a, R.ood_trace_z[c]);
        fe_to_bytes(e[W + c].a, R.ood_trace_zg[c]);
    }
    for (int j = 0; j < C; j++) fe_to_bytes(e[2 * W + j].a, R.ood_constraints[j]);
    uint8_t d[32];
    hash_elems(h.data(), 4 * W, d);
    coin.reseed(d);
    hash_elems(h.data() + 4 * W, 2 * C, d);
    coin.reseed(d);
}

DeepConstsE zk::draw_deep_consts_ext(Coin &coin, const std::vector<fe2> &e, int C, fe2 z, fe2 zg, zk_record &R) {
    DeepConstsE D;
    memset(&D, 0, sizeof D);
    fe2 k1 = fe2_zero(), k2 = fe2_zero();
    for (int c = 0; c < W; c++) {
        D.alpha_t[c] = coin.draw_ext(2);
        fe_to_bytes(D.alpha_t[c].a, R.deep_t[c]);
        k1 = fe2_add(k1, fe2_mul(D.alpha_t[c], e[c]));
        k2 = fe2_add(k2, fe2_mul(D.alpha_t[c], e[W + c]));
    }
    for (int j = 0; j < C; j++) {
        D.alpha_c[j] = coin.draw_ext(2);
        fe_to_bytes(D.alpha_c[j].a, R.deep_c[j]);
        k1 = fe2_add(k1, fe2_mul(D.alpha_c[j], e[2 * W + j]));
    }
    D.k1 = k1;
    D.k2 = k2;
    D.z = z;
    D.zg = zg;
    D.zb2 = fe_mul(z.b, z.b);
    D.zgb2 = fe_mul(zg.b, zg.b);
    return D;
}

FoldConstsE zk::fold_consts_ext(fe2 alpha, uint32_t fold) {
    const FoldConsts F1 = fold_consts(fe_zero(), fold);
    FoldConstsE F;
    memset(&F, 0, sizeof F);
    memcpy(F.zinv, F1.zinv, sizeof F.zinv);
    F.alpha = alpha;
    F.inv_offset = F1.inv_offset;
    F.inv_fold = F1.inv_fold;
    return F;
}

// rv: the last layer, planar (a plane then b plane, L values each, natural order over 3 * <w_L>)
int zk::remainder_step_ext(const std::vector<fe> &rv, uint32_t B, Coin &coin, zk_record &R, unsigned &degree_flag,
                           std::vector<fe> &rem_flat) {
    const size_t L = rv.size() / 2;
    std::vector<fe> va(rv.begin(), rv.begin() + L), vb(rv.begin() + L, rv.end());
    h_interp_coset3_cached(va);
    h_interp_coset3_cached(vb);
    const size_t rl = L / B;
    if (rl > ZK_MAX_REMAINDER) ZK_FAIL(ZK_ERR_INVALID_ARG, "remainder too large");
    for (size_t k = rl; k < L; k++)
        if (!fe_is_zero(va[k]) || !fe_is_zero(vb[k])) degree_flag = 1;
    R.remainder_len = (uint32_t)rl;
    rem_flat.clear();
    for (size_t k = 0; k < rl; k++) {
        fe_to_bytes(va[k], R.remainder[k]);
        rem_flat.push_back(va[k]);
        rem_flat.push_back(vb[k]);
    }
    hash_elems(rem_flat.data(), rem_flat.size(), R.remainder_commitment);
    coin.reseed(R.remainder_commitment);
    return ZK_OK;
}

static bool nonce_ok(const uint8_t seed[32], uint64_t nonce, uint32_t bits) {
    uint8_t d[32];
    Coin::merge_with_int(seed, nonce, d);
    uint64_t head;
    memcpy(&head, d, 8);
    const unsigned tz = head ? (unsigned)__builtin_ctzll(head) : 64;
    return tz >= bits;
}

int zk::grind_and_positions(zk_prover *p, Coin &coin, const zk_options *opt, size_t N, zk_record &R,
                            std::vector<uint64_t> &pos) {
    uint64_t nonce = 1;
    if (p && opt->grinding >= 8) {
        // ~2^grinding BLAKE3 calls: search batches of 2^22 nonces on the GPU, smallest hit wins
        if (!p->pow_seed) {
            ZK_CHECK_HIP(p->arena.alloc(&p->pow_seed, 8));
            ZK_CHECK_HIP(p->arena.alloc(&p->pow_best, 1));
        }
        ZK_TRY(h2d_small(p, p->pow_seed, coin.seed, 32));
        const unsigned long long none = ~0ULL;
        unsigned long long best = none;
        ZK_TRY(h2d_small(p, p->pow_best, &none, 8));
        const uint32_t batch = 1u << 22;
        for (uint64_t start = 1; best == none; start += batch) {
            grind_launch(p->st, p->pow_seed, start, batch, (int)opt->grinding, p->pow_best);
            ZK_TRY(d2h_small(p, &best, p->pow_best, 8));
            ZK_TRY(d2h_flush(p));
        }
        nonce = best;
        if (!nonce_ok(coin.seed, nonce, opt->grinding)) ZK_FAIL(ZK_ERR_DEVICE, "GPU grinding returned an invalid nonce");
    } else {
        while (!nonce_ok(coin.seed, nonce, opt->grinding)) nonce++;
    }
    R.pow_nonce = nonce;
    Coin::merge_with_int(coin.seed, nonce, coin.seed);
    coin.counter = 0;
    pos.clear();
    for (uint32_t q = 0; q < opt->num_queries; q++) {
        uint8_t d[32];
        coin.next(d);
        uint64_t v;
        memcpy(&v, d, 8);
        pos.push_back(v & (N - 1));
    }
    std::sort(pos.begin(), pos.end());
    pos.erase(std::unique(pos.begin(), pos.end()), pos.end());
    R.num_positions = (uint32_t)pos.size();
    memcpy(R.positions, pos.data(), pos.size() * 8);
    return ZK_OK;
}

std::vector<std::vector<uint64_t>> zk::fri_fold_positions(const std::vector<uint64_t> &pos, size_t N, uint32_t fold,
                                                          int nl) {
    std::vector<std::vector<uint64_t>> out(nl);
    std::vector<uint64_t> fp = pos;
    size_t dsz = N;
    for (int l = 0; l < nl; l++) {
        const size_t target = dsz / fold;
        std::vector<uint64_t> f;
        for (uint64_t x : fp) {
            const uint64_t q = x % target;
            if (std::find(f.begin(), f.end(), q) == f.end()) f.push_back(q);
        }
        out[l] = f;
        fp = f;
        dsz = target;
    }
    return out;
}

std::vector<uint8_t> zk::serialize_proof(size_t n, const zk_options *opt, int C, const zk_record &R, const fe *ood,
                                         const Openings &O, const std::vector<fe> *rem_flat) {
    std::vector<uint8_t> out;
    serialize_proof(n, opt, C, R, ood, O, rem_flat, out);
    return out;
}

void zk::serialize_proof(size_t n, const zk_options *opt, int C, const zk_record &R, const fe *ood, const Openings &O,
                         const std::vector<fe> *rem_flat, std::vector<uint8_t> &out) {
    const int nl = (int)R.num_fri_layers;
    const int K = (int)opt->field_extension, ES = 16 * K;
    const size_t nu = R.num_positions;
    Bytes pf;
    pf.v.swap(out);  // write into the caller's storage (capacity kept across proofs: no page faults)
    pf.v.clear();
    static thread_local Bytes paths;
    pf.u8(W);
    pf.u8(0);
    pf.u8(0);
    pf.u8((uint8_t)ilog2(n));
    pf.u16(0);
    pf.u8(16);
    pf.u64(ZK_P_LO);
    pf.u64(ZK_P_HI);
    pf.u8((uint8_t)opt->num_queries);
    pf.u8((uint8_t)opt->blowup);
    pf.u8((uint8_t)opt->grinding);
    pf.u8((uint8_t)opt->field_extension);
    pf.u8((uint8_t)opt->fri_folding);
    pf.u8((uint8_t)opt->fri_rem_max_deg);
    pf.u8((uint8_t)nu);
    pf.u16((uint16_t)(32 * (2 + nl + 1)));
    pf.put(R.trace_root, 32);
    pf.put(R.constraint_root, 32);
    for (int l = 0; l < nl; l++) pf.put(R.fri_roots[l], 32);
    pf.put(R.remainder_commitment, 32);
    auto write_queries = [&](const void *vals, size_t vlen, int b) {
        paths.v.clear();
        const BatchPlan &plan = O.plans[b];
        paths.u8((uint8_t)plan.paths.size());
        size_t k = 0;
        for (auto &path : plan.paths) {
            paths.u8((uint8_t)path.size());
            for (size_t t = 0; t < path.size(); t++, k++) paths.put(&O.digests[b][32 * k], 32);
        }
        pf.u32((uint32_t)vlen);
        pf.put(vals, vlen);
        pf.u32((uint32_t)paths.v.size());
        pf.put(paths.v.data(), paths.v.size());
    };
    pf.u8(1);
    write_queries(O.trace_rows.data(), nu * W * 16, 0);
    write_queries(O.comp_rows.data(), nu * C * ES, 1);
    pf.u16((uint16_t)(1 + 2 * W * ES));
    pf.u8(2);
    for (int c = 0; c < W; c++) {
        pf.put(&ood[c * K], ES);
        pf.put(&ood[(W + c) * K], ES);
    }
    pf.u16((uint16_t)(C * ES));
    pf.put(ood + 2 * W * K, C * ES);
    pf.u8((uint8_t)nl);
    for (int l = 0; l < nl; l++) write_queries(O.fri_rows[l].data(), O.fri_rows[l].size() * 16, 2 + l);
    pf.u16((uint16_t)(R.remainder_len * ES));
    if (rem_flat) pf.put(rem_flat->data(), R.remainder_len * ES);
    else pf.put(R.remainder, R.remainder_len * 16);
    pf.u8(0);
    pf.u64(R.pow_nonce);
    pf.u8(0);
    out.swap(pf.v);
}

int zk::deliver_proof(const std::vector<uint8_t> &bytes, unsigned degree_flag, uint8_t *proof_out, size_t *proof_len) {
    int status = degree_flag ? ZK_ERR_DEGREE : ZK_OK;
    if (degree_flag) g_err = "the trace does not satisfy ProcessorAir (composition degree check failed)";
    if (proof_out && *proof_len >= bytes.size())
        memcpy(proof_out, bytes.data(), bytes.size());
    else if (status == ZK_OK) {
        status = ZK_ERR_BUFFER_TOO_SMALL;
        g_err = "proof buffer too small";
    }
    *proof_len = bytes.size();
    return status;
}

// ---------------------------------------------------------------- the single-GPU prove path
// Coset LDE of the ncols column polynomials at `polys` into the coset-major `lde` and the commitment to
// its rows (leaves, nodes; the root is read back with the caller's next d2h_flush).
static int lde_commit(zk_prover *p, Plan *pl, const fe *polys, int ncols, fe *lde, uint8_t *leaves, uint8_t *nodes,
                      uint8_t root[32]) {
    const int log_n = pl->log_n, log_b = pl->log_b;
    const size_t n = (size_t)1 << log_n, B = (size_t)1 << log_b;
    ntt_lde(p->st, pl->Tn, pl->ct, polys, n, ncols, 0, 1, (int)B, lde, B * n, n, p->tmp);
    hash_rows_cosets(p->st, lde, ncols, log_n, log_b, 0, log_b, leaves);
    merkle_tree(p->st, leaves, n * B, nodes);
    return d2h_small(p, root, nodes + 32, 32);
}

// Where the trace comes from: resident in HBM (zk_prove_device), or W host columns (zk_prove,
// zk_prove_columns, zk_lde_new: the reference's TraceTable / ColMatrix, vm/src/lib.rs:18, 26).
struct TraceSrc {
    const fe *dev = nullptr;
    const uint8_t *const *cols = nullptr;
    const FixedCols *fixed = nullptr;  // with dev: only the dynamic columns are in dev (zk_vm_prove)
    bool hint_ok = true;               // host columns: the sparse hint of the previous proof may be used
    bool no_virtual = false;           // every trace LDE column written (stage dumps read them)
    const uint8_t *key = nullptr;      // host columns: the program hash the hints are keyed by (with n)
};

// The hint set of (n, program), or null (prover state: zk_prover::HintSet)
static zk_prover::HintSet *hint_find(zk_prover *p, size_t n, const uint8_t *key) {
    if (!key) return nullptr;
    for (auto &h : p->hint_sets)
        if (h.n == n && !memcmp(h.key, key, 32)) return &h;
    return nullptr;
}
// ... found or made, evicting the least recently used set
static zk_prover::HintSet *hint_slot(zk_prover *p, size_t n, const uint8_t *key) {
    zk_prover::HintSet *h = hint_find(p, n, key);
    if (h) return h;
    h = &p->hint_sets[0];
    for (auto &e : p->hint_sets)
        if (e.used < h->used) h = &e;
    *h = zk_prover::HintSet{};
    h->n = n;
    memcpy(h->key, key, 32);
    return h;
}

// Virtual columns: the first trace column no transition constraint or assertion reads -- the evaluator reads columns
// 0 .. 12 + 2 lwe_size - 1 <= 21 (enforce_add2 reads 2 lwe_size stack items, lwe_size <= 5; constrains.rs) -- so a
// hinted sparse column from here on needs no LDE in memory (ZK_VIRTUAL=0 writes it)
constexpr int ZK_VIRT_MIN_COL = 22;
static bool virtual_on() {
    static const bool on = [] {
        const char *e = getenv("ZK_VIRTUAL");
        return !(e && !strcmp(e, "0"));
    }();
    return on;
}

// Column groups of a host-resident trace upload.  The copy engine streams group g + 1 while the CUs interpolate and
// extend group g; more groups overlap more of the copy but add a launch drain per NTT pass and group.  A/B on one box
// (3 provers in flight): 1 group 12.73-13.02 ms per proof at 22.7 ms latency, 2 groups 13.15-13.24 / 18.7, 4 groups
// 13.16-13.32 / 16.8, 7 groups of 4 13.02-13.04 / 15.9 (device-resident 12.15-12.32).  Round 4: the rows are hashed
// block by block as their columns' LDEs complete (hash_rows_blocks: a 28-element row is 7 BLAKE3 blocks of 4
// columns), and the last 4 columns go up as two groups of 2, so after the last copy only 2 columns' NTTs, one
// compression per row and the Merkle tree remain (latency 15.3-15.4 -> 13.9-14.2 ms against 7 groups of 4, all rows
// hashed at the end; profiles/r04_ab_queues_pass1.txt).

// hipMemcpyAsync from page-locked memory (zk_host_alloc, zk_host_register, any hipHostMalloc'd or
// hipHostRegister'ed buffer) is a DMA in stream order; from pageable memory the runtime stages the copy
// through its own pinned buffers and returns once the source has been read (the host thread copies).
// Both are correct here; the pinned form is the fast one (DESIGN.md "Host-resident trace").
// Columns that are contiguous in host memory (zk_prove's single buffer) go up as one copy per run.
static int upload_trace_group(zk_prover *p, const TraceSrc &src, size_t n, int c0, int nc) {
    const size_t col = n * sizeof(fe);
    p->up_bytes += (uint64_t)nc * col;
    for (int c = c0; c < c0 + nc;) {
        int e = c + 1;
        while (e < c0 + nc && src.cols[e] == src.cols[e - 1] + col) e++;
        ZK_CHECK_HIP(hipMemcpyAsync(p->d_trace + (size_t)c * n, src.cols[c], (size_t)(e - c) * col, hipMemcpyHostToDevice,
                                    p->up));
        c = e;
    }
    return ZK_OK;
}

// S2: interpolate the 28 trace columns (winter-math interpolate_poly over <w_n>), extend them over the B
// cosets of the LDE domain (coset r: the coefficients scaled by (3 w_N^r)^k) and commit to the rows.
// A host-resident trace goes up on the upload stream in the column groups of the upload plan; each group's
// event gates that group's interpolation and coset LDE on the compute stream.
// Sparse trace columns (SparseCols): a column that is zero in every row but the last (the VM's stack registers past
// the program's maximum depth, five of the benchmark's 28) interpolates to last * lagr and extends to last * lagr_lde;
// sparse_detect flags them on the device and the NTT passes skip their DFTs.  Exact: the same polynomials and LDE.
// ZK_SPARSE=0 transforms every column.
bool zk::sparse_on() {
    static const bool on = [] {
        const char *e = getenv("ZK_SPARSE");
        return !(e && !strcmp(e, "0"));
    }();
    return on;
}

// Narrow columns (host-resident traces): ZK_NARROW=0 uploads every column whole.
bool zk::narrow_on() {
    static const bool on = [] {
        const char *e = getenv("ZK_NARROW");
        return !(e && !strcmp(e, "0"));
    }();
    return on;
}

// The AIR clock (ZK_CLOCK=0 turns its derivation off)
bool zk::clock_on() {
    static const bool on = [] {
        const char *e = getenv("ZK_CLOCK");
        return !(e && !strcmp(e, "0"));
    }();
    return on;
}

int zk::plan_rank_tables(zk_prover *p, Plan *pl, int r0, int G) {
    if (p->shard_world <= 1 || !pl->lagr) return ZK_OK;  // a full prover's tables hold every coset
    const size_t n = (size_t)1 << pl->log_n, Bl = ((size_t)1 << pl->log_b) >> ilog2((size_t)G);
    // the rank's block of cosets r0 .. r0 + Bl - 1 (shard.hip: rank g owns g Bl + j)
    if (pl->lagr_lde && pl->lde_r0 == r0 && pl->lde_shift == 0 && pl->lde_cos == (int)Bl) return ZK_OK;
    if (!pl->lagr_lde) ZK_CHECK_HIP(p->arena.alloc(&pl->lagr_lde, Bl * n));
    ntt_lde(p->st, pl->Tn, pl->ct, pl->lagr, n, 1, r0, 1, (int)Bl, pl->lagr_lde, Bl * n, n, p->tmp);
    if (pl->id_lde) ntt_lde(p->st, pl->Tn, pl->ct, pl->id_poly, n, 1, r0, 1, (int)Bl, pl->id_lde, Bl * n, n, p->tmp);
    pl->lde_r0 = r0;
    pl->lde_shift = 0;
    pl->lde_cos = (int)Bl;
    ZK_CHECK_HIP(hipStreamSynchronize(p->st));
    return ZK_OK;
}

// the identity column 0, 1, ..., n-1 interpolated and extended over the cosets the plan's fill tables hold
// (Plan::id_poly / id_lde, lde_r0 / lde_shift / lde_cos: all B for a full prover), once per plan
int zk::clock_tables(zk_prover *p, Plan *pl) {
    if (pl->id_poly) return ZK_OK;
    if (!pl->lde_cos) ZK_FAIL(ZK_ERR_INVALID_ARG, "internal error: the plan's rank tables are not built");
    const size_t n = (size_t)1 << pl->log_n, nc = (size_t)pl->lde_cos;
    fe *poly = nullptr, *lde = nullptr;
    ZK_CHECK_HIP(p->arena.alloc(&poly, n));
    ZK_CHECK_HIP(p->arena.alloc(&lde, nc * n));
    std::vector<fe> id(n);
    for (size_t i = 0; i < n; i++) id[i] = fe_make(i);
    fe *d = nullptr;
    ZK_CHECK_HIP(hipMalloc(&d, n * sizeof(fe)));
    hipError_t err = hipMemcpy(d, id.data(), n * sizeof(fe), hipMemcpyHostToDevice);
    if (err == hipSuccess) {
        const fe inv_n = h_inv(fe_make(n));
        ntt(p->st, pl->Tn, d, n, poly, n, 1, true, nullptr, &inv_n, p->tmp);
        ntt_lde(p->st, pl->Tn, pl->ct, poly, n, 1, pl->lde_r0, 1 << pl->lde_shift, (int)nc, lde, nc * n, n, p->tmp);
        err = hipStreamSynchronize(p->st);
    }
    (void)hipFree(d);
    ZK_CHECK_HIP(err);
    pl->id_poly = poly;
    pl->id_lde = lde;
    return ZK_OK;
}

// rows [r0, r1) of a host column: row i holds i (the AIR clock)
bool zk::clock_rows(const uint8_t *col, size_t r0, size_t r1) {
    const uint64_t *v = reinterpret_cast<const uint64_t *>(col);
    uint64_t bad = 0;
    for (size_t i = r0; i < r1; i++) bad |= (v[2 * i] ^ (uint64_t)i) | v[2 * i + 1];
    return bad == 0;
}

// rows [r0, r1) of a host column as `width`-byte integers (1 or 4) at dst + width * row; false if a value does not fit
bool zk::pack_rows(const uint8_t *col, size_t r0, size_t r1, int width, uint8_t *dst) {
    const uint64_t *v = reinterpret_cast<const uint64_t *>(col);
    uint64_t over = 0;
    if (width == 1) {
        for (size_t i = r0; i < r1; i++) {
            const uint64_t lo = v[2 * i], hi = v[2 * i + 1];
            over |= (lo >> 8) | hi;
            dst[i] = (uint8_t)lo;
        }
    } else {
        uint32_t *d = reinterpret_cast<uint32_t *>(dst);
        for (size_t i = r0; i < r1; i++) {
            const uint64_t lo = v[2 * i], hi = v[2 * i + 1];
            over |= (lo >> 32) | hi;
            d[i] = (uint32_t)lo;
        }
    }
    return over == 0;
}

// rows [r0, r1) of a host column all zero
bool zk::zero_rows(const uint8_t *col, size_t r0, size_t r1) {
    const uint64_t *v = reinterpret_cast<const uint64_t *>(col);
    uint64_t any = 0;
    for (size_t i = 2 * r0; i < 2 * r1; i++) any |= v[i];
    return any == 0;
}

int zk::sparse_begin(zk_prover *p, Plan *pl, SparseCols *out, const SparseCols **sp) {
    *sp = nullptr;
    if (!sparse_on() || !pl->lagr || !pl->lagr_lde) return ZK_OK;
    if (!p->sp_nz) {
        ZK_CHECK_HIP(p->arena.alloc(&p->sp_nz, 4 * W));  // nonzero, 8-bit, 32-bit flags; [3W]: column 0 not the clock
        ZK_CHECK_HIP(p->arena.alloc(&p->sp_last, W));
        ZK_CHECK_HIP(hipHostMalloc((void **)&p->sp_h, 3 * W * sizeof(unsigned), hipHostMallocDefault));
    }
    ZK_CHECK_HIP(hipMemsetAsync(p->sp_nz, 0, 4 * W * sizeof(unsigned), p->st));
    *out = SparseCols{p->sp_nz, p->sp_last, pl->lagr, pl->lagr_lde, 0};
    out->lde_r0 = pl->lde_r0;
    out->lde_shift = pl->lde_shift;
    if (clock_on()) {  // the AIR clock of column 0, detected with the sparse columns (device-side traces)
        ZK_TRY(clock_tables(p, pl));
        out->id_poly = pl->id_poly;
        out->id_lde = pl->id_lde;
        out->idoff = 3 * W;
    }
    *sp = out;
    return ZK_OK;
}

static int trace_lde_commit(zk_prover *p, Plan *pl, const TraceSrc &src, size_t n, uint8_t root[32]) {
    const fe inv_n = h_inv(fe_make(n));
    p->virt = 0;  // every LDE column is written unless the host path below takes some as virtual
    SparseCols spc{};
    const SparseCols *sp = nullptr;
    if (!src.fixed) ZK_TRY(sparse_begin(p, pl, &spc, &sp));
    p->sp_used = sp != nullptr;
    if (src.dev && src.fixed) {
        // zk_vm_prove: interpolate and extend the dynamic stack columns only; the preprocessed ones by one pass
        const FixedCols &fx = *src.fixed;
        const size_t B = (size_t)1 << pl->log_b, c0 = 12;
        if (fx.md > 0) {
            ntt(p->st, pl->Tn, src.dev + c0 * n, n, p->polys + c0 * n, n, fx.md, true, nullptr, &inv_n, p->tmp);
            ntt_lde(p->st, pl->Tn, pl->ct, p->polys + c0 * n, n, fx.md, 0, 1, (int)B, p->lde + c0 * B * n, B * n, n,
                    p->tmp);
        }
        const int pre = p->fix_prefix_blocks;  // (zk_vm_prove: the preprocessed part went first, fixed_prefix)
        p->fix_prefix_blocks = 0;
        if (pre) {
            hash_rows_blocks(p->st, p->lde, W, pl->log_n, pl->log_b, pre, W / 4, p->leaves);
        } else {
            if (!p->fix_ws) ZK_CHECK_HIP(p->arena.alloc(&p->fix_ws, W));
            fe_ws ws[W];
            for (int c = 0; c < W; c++) ws[c] = make_fe_ws(fx.last[c]);
            ZK_TRY(h2d_small(p, p->fix_ws, ws, sizeof ws));
            fixed_axpy(p->st, fx, p->fix_ws, n, B, p->polys, p->lde);
            hash_rows_cosets(p->st, p->lde, W, pl->log_n, pl->log_b, 0, pl->log_b, p->leaves);
        }
        merkle_tree(p->st, p->leaves, n * B, p->nodes);
        return d2h_small(p, root, p->nodes + 32, 32);
    }
    if (src.dev) {
        if (sp) sparse_detect(p->st, src.dev, n, 0, W, *sp);
        ntt(p->st, pl->Tn, src.dev, n, p->polys, n, W, true, nullptr, &inv_n, p->tmp, sp);
        const size_t B = (size_t)1 << pl->log_b;
        ntt_lde(p->st, pl->Tn, pl->ct, p->polys, n, W, 0, 1, (int)B, p->lde, B * n, n, p->tmp, sp);
        hash_rows_cosets(p->st, p->lde, W, pl->log_n, pl->log_b, 0, pl->log_b, p->leaves);
        merkle_tree(p->st, p->leaves, n * B, p->nodes);
        return d2h_small(p, root, p->nodes + 32, 32);
    }
    const int log_n = pl->log_n, log_b = pl->log_b;
    const size_t B = (size_t)1 << log_b;
    // The device trace buffer is free: the previous proof on this prover returned only after its stream drained
    // (and the trace is read by the interpolation alone).
    // hints of the previous proof of this length (hint_ok: prove_impl allows them): its sparse columns (zero but the
    // last row: nothing goes up but that value), and its narrow ones (8- or 32-bit values before the last row), which
    // go up packed.  Host threads check every hinted value while the other columns go up: a narrow column that does
    // not fit goes up whole, a sparse one that is not sparse voids the proof (prove_impl redoes it without hints).
    const zk_prover::HintSet *H = sp && src.hint_ok ? hint_find(p, n, src.key) : nullptr;
    const bool fresh = H && H->have;
    const uint32_t hint = fresh ? H->sparse : 0u;
    const uint32_t nw8 = fresh && narrow_on() ? H->nw8 & ~hint : 0u;
    uint32_t nw32 = fresh && narrow_on() ? H->nw32 & ~hint & ~nw8 : 0u;
    // The AIR clock: constraint 0 (clk' = clk + 1, air/src/constrains.rs) and the assertion clk[0] = 0 force rows
    // 0 .. n-2 of column 0 of any trace the AIR accepts to 0 .. n-2, so its interpolant and LDE are the identity
    // column's (per plan) plus (last - (n - 1)) times e_(n-1)'s: no upload, no transform.  Taken once the previous
    // proof found column 0 narrow (32-bit), checked by host threads while the other columns go up; a column that is
    // not 0 .. n-2 voids the proof, which is redone without hints (and this length is not speculated again).
    const bool clk = fresh && clock_on() && (nw32 & 1u) && !H->clk_off;
    if (clk) nw32 &= ~1u;
    p->clk_used = clk;
    p->clk_bad = false;
    const uint32_t virt = !src.no_virtual && virtual_on() ? hint & ~((1u << ZK_VIRT_MIN_COL) - 1u) : 0u;
    p->virt = 0;  // (set once the hinted columns' last rows are on the device)
    p->sp_hinted = hint;
    p->up_bytes = 0;
    p->up_sparse = hint;
    p->up_nw8 = p->up_nw32 = 0;
    int dense[W], nd = 0, hin[W], nh = 0, nar[W], nn = 0;
    for (int c = 0; c < W; c++) {
        if (clk && c == 0) continue;
        if ((hint >> c) & 1u) hin[nh++] = c;
        else if (((nw8 | nw32) >> c) & 1u) nar[nn++] = c;
        else dense[nd++] = c;
    }
    if (sp) spc.wstride = W;  // width flags for the next proof's narrow hint
    bool ready[W] = {};
    // contiguous runs of a column list: f(first column, count)
    auto runs = [](const int *cols, int k, auto f) -> int {
        for (int i = 0; i < k;) {
            int j = i + 1;
            while (j < k && cols[j] == cols[j - 1] + 1) j++;
            ZK_TRY(f(cols[i], j - i));
            i = j;
        }
        return ZK_OK;
    };
    // with the hints learned, the uploaded columns' flags come from the interpolation's pass 1 (no separate pass over
    // them; a column found sparse there is transformed in full this time and hinted next time)
    const bool fuse_det = fresh;
    bool fused_tf = false, all_tf = false;
    auto transform = [&](int c0, int nc) -> int {  // interpolation + coset LDE of columns [c0, c0 + nc)
        SparseCols gsp = spc;
        gsp.col0 = c0;
        gsp.fused = fused_tf;
        gsp.all = all_tf;
        ntt(p->st, pl->Tn, p->d_trace + (size_t)c0 * n, n, p->polys + (size_t)c0 * n, n, nc, true, nullptr, &inv_n, p->tmp,
            sp ? &gsp : nullptr);
        ntt_lde(p->st, pl->Tn, pl->ct, p->polys + (size_t)c0 * n, n, nc, 0, 1, (int)B, p->lde + (size_t)c0 * B * n, B * n, n,
                p->tmp, sp ? &gsp : nullptr);
        return ZK_OK;
    };
    int hashed = 0;
    auto hash_ready = [&](bool last) {  // the blocks whose 4 columns are extended, at least two per launch but the last
        int b = hashed;
        while (b < W / 4 && ready[4 * b] && ready[4 * b + 1] && ready[4 * b + 2] && ready[4 * b + 3]) b++;
        if (b - hashed >= 2 || (last && b > hashed)) {
            hash_rows_blocks(p->st, p->lde, W, log_n, log_b, hashed, b, p->leaves,
                             VirtCols{p->virt, p->sp_last, pl->lagr_lde});
            hashed = b;
        }
    };
    // the kernels of an uploaded column list: detection (flags for the next proof's hints), transforms, hashing
    auto process = [&](const int *cols, int nc) -> int {
        if (sp && !fuse_det)
            ZK_TRY(runs(cols, nc, [&](int c0, int k) { sparse_detect(p->st, p->d_trace, n, c0, k, spc); return ZK_OK; }));
        fused_tf = sp && fuse_det;
        const int rc = runs(cols, nc, transform);
        fused_tf = false;
        ZK_TRY(rc);
        for (int i = 0; i < nc; i++) ready[cols[i]] = true;
        hash_ready(false);
        return ZK_OK;
    };
    // host checks of the hints: one pool task per quarter million rows of a hinted column, the narrow ones packing
    // rows 0 .. n-2 (1 or 4 bytes each) into pinned h_pack as they go; the latch is waited for on every way out (the
    // tasks read the caller's columns)
    NarrowCols NC{};
    size_t pack_bytes = 0;
    for (int i = 0; i < nn; i++) {
        NC.col[i] = nar[i];
        NC.width[i] = ((nw8 >> nar[i]) & 1u) ? 1 : 4;
        NC.off[i] = pack_bytes;
        pack_bytes += ((size_t)NC.width[i] * n + 15) & ~(size_t)15;
    }
    NC.count = nn;
    std::atomic<uint32_t> pack_bad{0}, sparse_bad{0}, clock_bad{0};
    // Two upload schedules (set per proof by prove_once, see zk_prover::lat_sched):
    //  - throughput (other proofs in flight on the device): the narrow columns go up in two parts (the first half of
    //    them, the rest) through the copy engine, each as soon as its packing is done, in quarter-million-row tasks;
    //  - latency (this proof alone on the device): dense groups 0 and 1 start crossing the link at once; the narrow
    //    columns are packed in parts of 1, 2, 2, ... columns (64 K-row tasks, so each part is ready in ~0.1-0.2 ms)
    //    and each part's expansion kernel reads the pinned packed bytes itself (no copy engine: that is busy with the
    //    dense groups), so the first kernels start ~0.2 ms into the call and the device has the narrow columns' work
    //    while the first dense groups cross.
    const bool lat = p->lat_sched && nn > 0;
    int pb[W + 1], np = 0;  // part k: narrow columns pb[k] .. pb[k+1]-1
    pb[0] = 0;
    if (lat) {
        for (int i = 0; i < nn;) {
            i = std::min(nn, i + (np == 0 ? 1 : 2));
            pb[++np] = i;
        }
    } else if (nn) {
        pb[1] = (nn + 1) / 2;
        pb[2] = nn;
        np = pb[1] < nn ? 2 : 1;
    }
    Latch packed[W], checked, clocked;
    struct PackWait {
        Latch *parts;
        const int &np;
        Latch &b, &c;
        ~PackWait() {
            for (int k = 0; k < np; k++) parts[k].wait();
            b.wait();
            c.wait();
        }
    } pack_wait{packed, np, checked, clocked};
    constexpr size_t R = (size_t)1 << 18;
    const size_t per = (n - 1 + R - 1) / R;
    const size_t Rp = lat ? (size_t)1 << 16 : R, perp = (n - 1 + Rp - 1) / Rp;  // packing task rows
    if (nn) {
        if (pack_bytes > p->h_pack_cap) {  // the previous proof's copies from it have drained (CopyGuard)
            if (p->h_pack) (void)hipHostFree(p->h_pack);
            p->h_pack = nullptr;
            p->h_pack_cap = 0;
            ZK_CHECK_HIP(hipHostMalloc((void **)&p->h_pack, pack_bytes, hipHostMallocMapped | hipHostMallocCoherent));
            p->h_pack_cap = pack_bytes;
        }
        for (int k = 0; k < np; k++) packed[k].reset((int)(perp * (pb[k + 1] - pb[k])));
        for (int i = 0, k = 0; i < nn; i++) {
            if (i == pb[k + 1]) k++;  // part k holds narrow column i
            for (size_t t = 0; t < perp; t++) {
                const size_t r0 = t * Rp, r1 = std::min(n - 1, r0 + Rp);
                const uint8_t *col = src.cols[nar[i]];
                uint8_t *dst = p->h_pack + NC.off[i];
                const int width = NC.width[i], c = nar[i];
                const bool tail = r1 == n - 1;
                Latch *lt = &packed[k];
                HostPool::get().submit([=, &pack_bad] {
                    if (!pack_rows(col, r0, r1, width, dst)) pack_bad.fetch_or(1u << c);
                    if (tail) memset(dst + (size_t)width * (n - 1), 0, width);  // the last row's slot (not read)
                    lt->count_down();
                });
            }
        }
    }
    if (nh) {
        checked.reset((int)(per * nh));
        for (int i = 0; i < nh; i++)
            for (size_t t = 0; t < per; t++) {
                const size_t r0 = t * R, r1 = std::min(n - 1, r0 + R);
                const uint8_t *col = src.cols[hin[i]];
                const int c = hin[i];
                HostPool::get().submit([=, &sparse_bad, &checked] {
                    if (!zero_rows(col, r0, r1)) sparse_bad.fetch_or(1u << c);
                    checked.count_down();
                });
            }
        // hinted sparse columns: their coefficients and LDE are last * e_(n-1)'s (the NTT passes' sparse fill)
        fe lastv[W];
        memset(lastv, 0, sizeof lastv);
        for (int i = 0; i < nh; i++) memcpy(&lastv[hin[i]], src.cols[hin[i]] + (n - 1) * sizeof(fe), sizeof(fe));
        ZK_TRY(h2d_small(p, p->sp_last, lastv, sizeof lastv));
        // no transform: the fills alone -- the coefficients of every hinted column, the LDE of the non-virtual ones
        int hnv[W], nhv = 0;
        for (int i = 0; i < nh; i++)
            if (!((virt >> hin[i]) & 1u)) hnv[nhv++] = hin[i];
        SparseCols gsp = spc;
        gsp.fused = false;
        gsp.all = true;
        ZK_TRY(runs(hin, nh, [&](int c0, int nc) {
            gsp.col0 = c0;
            ntt(p->st, pl->Tn, p->d_trace + (size_t)c0 * n, n, p->polys + (size_t)c0 * n, n, nc, true, nullptr, &inv_n,
                p->tmp, &gsp);
            return ZK_OK;
        }));
        ZK_TRY(runs(hnv, nhv, [&](int c0, int nc) {
            gsp.col0 = c0;
            ntt_lde(p->st, pl->Tn, pl->ct, p->polys + (size_t)c0 * n, n, nc, 0, 1, (int)B, p->lde + (size_t)c0 * B * n,
                    B * n, n, p->tmp, &gsp);
            return ZK_OK;
        }));
        p->virt = virt;
        memcpy(p->virt_last, lastv, sizeof lastv);
        p->virt_lagr = pl->lagr_lde;
        for (int i = 0; i < nh; i++) ready[hin[i]] = true;
    }
    if (clk) {
        ZK_TRY(clock_tables(p, pl));
        clocked.reset((int)per);
        const uint8_t *col = src.cols[0];
        for (size_t t = 0; t < per; t++) {
            const size_t r0 = t * R, r1 = std::min(n - 1, r0 + R);
            HostPool::get().submit([=, &clock_bad, &clocked] {
                if (!clock_rows(col, r0, r1)) clock_bad.store(1u);
                clocked.count_down();
            });
        }
        fe last0;
        memcpy(&last0, col + (n - 1) * sizeof(fe), sizeof(fe));
        const fe_ws d = make_fe_ws(fe_sub(last0, fe_make(n - 1)));
        axpy_fill(p->st, pl->id_poly, pl->lagr, d, n, p->polys);
        axpy_fill(p->st, pl->id_lde, pl->lagr_lde, d, B * n, p->lde);
        ready[0] = true;
    }
    // Upload items, each one copy (or a run of column copies) and an event on the shared upload stream: the wide
    // columns in groups of 4, the last 4 as 2 + 2 (after the last copy only 2 columns' NTTs, the last hash blocks and
    // the Merkle tree remain); the packed narrow columns first, in two parts (below); narrow columns that did not fit,
    // whole, last.  The next item's copy is queued before the host waits for the current one's event
    // (the compute stream never parks on the upload stream: a parked stream would hold up the kernels of other
    // provers that share its hardware queue), so the copy engine always has the next group.
    int gsz[W], ngroups = 0;
    // (a first group of 1 or 2 columns, so the first kernels start after a shorter copy, measured slower: latency
    // 13.90-13.95 vs 13.73-13.79 ms, throughput unchanged; profiles/r04h_ab_first_group.txt; round 5, 3 x 31 single
    // calls: 14.75-14.78 / 14.67-14.70 vs 14.76-14.84 ms, profiles/r05d_latency_ab.txt)
    int left = nd;
    while (left > 0) {
        const int k = left > 4 ? 4 : left > 2 ? 2 : left;
        gsz[ngroups++] = left == 4 ? 2 : k;
        left -= gsz[ngroups - 1];
    }
    if (ngroups + (lat ? 1 : np + 1) > ZK_UPLOAD_GROUPS_MAX) ZK_FAIL(ZK_ERR_INVALID_ARG, "too many upload groups");
    struct Item {
        const int *cols = nullptr;
        int nc = 0;
        int part = -1;  // narrow part (packed), or -1 (whole columns)
        int ev = 0;
    };
    int fallback[W], nfb = 0, good[W], ev = 0, gi = 0, di = 0;
    bool narrow_done[2] = {np < 1, np < 2}, fb_done = false;
    NarrowCols G[W] = {};
    size_t part_off[W + 1];  // byte range of each part in h_pack
    for (int k = 0; k <= np; k++) part_off[k] = pb[k] < nn ? NC.off[pb[k]] : pack_bytes;
    uint8_t *stage = reinterpret_cast<uint8_t *>(p->ctmp);  // composition scratch: free until S4
    // part k's columns once packed (the host waits for its packing), its unpackable ones to the fallback list
    auto narrow_item = [&](int k, Item *it) -> bool {
        packed[k].wait();
        if (k < 2) narrow_done[k] = true;
        const uint32_t bad = pack_bad.load();
        NarrowCols &g = G[k];
        int *gd = good + pb[k], ng = 0;
        for (int i = pb[k]; i < pb[k + 1]; i++) {
            if ((bad >> nar[i]) & 1u) {  // a value that does not fit: this column goes up whole
                fallback[nfb++] = nar[i];
                continue;
            }
            g.col[g.count] = nar[i];
            g.width[g.count] = NC.width[i];
            g.off[g.count] = NC.off[i];
            memcpy(&g.last[g.count], src.cols[nar[i]] + (n - 1) * sizeof(fe), sizeof(fe));
            g.count++;
            gd[ng++] = nar[i];
        }
        if (!ng) return false;
        *it = Item{gd, ng, k, -1};
        return true;
    };
    auto count_part = [&](int k) {  // part k's packed bytes cross the link
        p->up_bytes += part_off[k + 1] - part_off[k];
        const NarrowCols &g = G[k];
        for (int i = 0; i < g.count; i++) (g.width[i] == 1 ? p->up_nw8 : p->up_nw32) |= 1u << g.col[i];
    };
    auto issue = [&](const Item &it) -> int {
        std::lock_guard<std::mutex> lk(*p->up_mu);
        // a copy that fails part-way through the item still gets the item's event behind the copies queued before
        // it, so upload_drain (CopyGuard) waits for every DMA that reads the caller's columns
        UploadEvent rec{p->ev_up[it.ev], p->up};
        if (it.part >= 0) {
            const size_t a = part_off[it.part];
            ZK_CHECK_HIP(hipMemcpyAsync(stage + a, p->h_pack + a, part_off[it.part + 1] - a, hipMemcpyHostToDevice,
                                        p->up));
            count_part(it.part);
        } else {
            ZK_TRY(runs(it.cols, it.nc, [&](int c0, int k) { return upload_trace_group(p, src, n, c0, k); }));
        }
        return rec.record();
    };
    if (lat) {
        // the latency schedule: dense groups 0 and 1 go up at once, group g + 2 once group g has landed; the narrow
        // parts in order as they are packed, each expanded straight from the pinned buffer; then the dense groups
        int gev[W];
        auto issue_dense = [&]() -> int {
            if (gi >= ngroups) return ZK_OK;
            gev[gi] = ev++;
            const Item d{dense + di, gsz[gi], -1, gev[gi]};
            di += gsz[gi++];
            return issue(d);
        };
        ZK_TRY(issue_dense());
        ZK_TRY(issue_dense());
        // (h_pack is pinned and mapped; part k's bytes are written by the pool threads before packed[k] opens and the
        // expansion kernel is launched after that, and a kernel dispatch acquires at system scope, so the kernel
        // reads this proof's bytes -- tests/test_gpu_parity.py changes a narrow column between proofs on this path)
        uint8_t *hp = nullptr;
        ZK_CHECK_HIP(hipHostGetDevicePointer((void **)&hp, p->h_pack, 0));
        for (int k = 0; k < np; k++) {
            Item it;
            if (!narrow_item(k, &it)) continue;
            count_part(k);
            expand_narrow(p->st, hp, G[k], n, p->d_trace);
            ZK_TRY(process(it.cols, it.nc));
        }
        for (int g = 0, d0 = 0; g < ngroups; d0 += gsz[g++]) {
            ZK_CHECK_HIP(hipEventSynchronize(p->ev_up[gev[g]]));
            ZK_TRY(issue_dense());
            ZK_TRY(process(dense + d0, gsz[g]));
        }
        narrow_done[0] = narrow_done[1] = true;  // (the fallback columns, if any, go through the loop below)
    }
    // The throughput schedule: the first narrow part before anything else (packed by the host threads in ~0.3 ms, a
    // few MB over PCIe: the first kernels start then instead of after a 64-MB dense group; one call alone -0.45 ms,
    // 14.32-14.36 vs 14.76-14.84 ms over 3 x 31 calls, profiles/r05d_latency_ab.txt), the second as soon as it is
    // packed, the dense groups in between.
    auto next_item = [&](Item *it) -> bool {
        if (!narrow_done[0] && narrow_item(0, it)) {
            it->ev = ev++;
            return true;
        }
        if (!narrow_done[1] && (packed[1].ready() || gi == ngroups) && narrow_item(1, it)) {
            it->ev = ev++;
            return true;
        }
        if (gi < ngroups) {
            *it = Item{dense + di, gsz[gi], -1, ev++};
            di += gsz[gi++];
            return true;
        }
        if (narrow_done[0] && narrow_done[1] && nfb && !fb_done) {
            fb_done = true;
            *it = Item{fallback, nfb, -1, ev++};
            return true;
        }
        return false;
    };
    Item cur;
    bool have = next_item(&cur);
    if (have) ZK_TRY(issue(cur));
    while (have) {
        Item nxt;
        const bool more = next_item(&nxt);
        if (more) ZK_TRY(issue(nxt));
        ZK_CHECK_HIP(hipEventSynchronize(p->ev_up[cur.ev]));
        if (cur.part >= 0) expand_narrow(p->st, stage, G[cur.part], n, p->d_trace);
        ZK_TRY(process(cur.cols, cur.nc));
        cur = nxt;
        have = more;
    }
    hash_ready(true);
    merkle_tree(p->st, p->leaves, n * B, p->nodes);
    if (sp) ZK_TRY(d2h_small(p, p->sp_h, p->sp_nz, 3 * W * sizeof(unsigned)));  // for the next proof's hints
    checked.wait();
    clocked.wait();
    p->sp_bad = sparse_bad.load();
    p->clk_bad = clock_bad.load() != 0;
    return d2h_small(p, root, p->nodes + 32, 32);
}

static void coset_major_rows_to_host(zk_prover *p, const fe *base, int ncols, size_t n, uint32_t B, uint8_t *dst) {
    // dst: N x ncols row-major (natural index)
    size_t N = n * B;
    std::vector<fe> h((size_t)ncols * N);
    (void)hipMemcpy(h.data(), base, h.size() * sizeof(fe), hipMemcpyDeviceToHost);
    fe *o = reinterpret_cast<fe *>(dst);
    for (int c = 0; c < ncols; c++)
        for (size_t i = 0; i < N; i++) o[i * ncols + c] = h[((size_t)c * B + (i % B)) * n + i / B];
}

// FieldExtension::Quadratic buffers (planar E): composition 2 x 8n, its inverse NTT, the composition LDE
// (up to 2 x 8 base columns), DEEP 2N, FRI layers 2(N + 16), OOD tables and partial sums.
int zk::ensure_ext(zk_prover *p) {
    if (p->x_comp) return ZK_OK;
    const size_t n = p->max_n, N = n * p->max_b, CE = 8 * n;
    const size_t Nl = p->shard_world ? N / (size_t)p->shard_world : N;  // LDE points held (see create_prover)
    DeviceArena &A = p->arena;
    ZK_CHECK_HIP(A.alloc(&p->x_comp, 2 * CE));
    ZK_CHECK_HIP(A.alloc(&p->x_ctmp, 2 * CE));
    ZK_CHECK_HIP(A.alloc(&p->x_clde, (size_t)2 * 8 * Nl));  // C <= 8 E columns
    ZK_CHECK_HIP(A.alloc(&p->x_deep, 2 * Nl));
    ZK_CHECK_HIP(A.alloc(&p->x_fri, 2 * (N + 16)));
    ZK_CHECK_HIP(A.alloc(&p->x_partials, (size_t)2 * (2 * ZK_MAX_COLS + ZK_MAX_CCOLS) * ood_waves(n)));
    ZK_CHECK_HIP(A.alloc(&p->x_tab, (size_t)2 * (128 + 2 * ood_waves(n))));
    ZK_CHECK_HIP(A.alloc((uint8_t **)&p->x_air, 2 * sizeof(AirConsts)));
    ZK_CHECK_HIP(A.alloc((uint8_t **)&p->x_deep_consts, sizeof(DeepConstsE)));
    ZK_CHECK_HIP(A.alloc((uint8_t **)&p->x_fold_consts, sizeof(FoldConstsE)));
    if (!p->shard_world) ZK_CHECK_HIP(A.alloc(&p->x_ulde, 2 * N));
    ZK_CHECK_HIP(A.alloc(&p->x_dscratch, 8 * (2048 + n / 2048 + 2) + 6 * n + 4 * (n / 256 + 1)));
    return ZK_OK;
}

// S4, shared by zk_prove_device and plug point 3 (build_constraint_commitment): interpolate the 8n
// composition values (coset-major in comp, KX planes) over the CE coset, split the polynomial into C
// column polynomials of n coefficients (p->cpolys; base column (c, j) of E column c at (c*KX + j)*n),
// extend them over the B LDE cosets into clde and commit to its rows (a leaf is C E values).
// p->flag is set when the interpolant has a coefficient at or beyond C*n (the degree check).
// bnd (KX coefficient planes, or nullptr when comp already holds the assertion terms): add the assertion
// terms' quotient polynomial to column 0 of each plane (boundary_poly_add) before the LDE.
// nce = 7 (C <= 7): only CE cosets 0..6 were evaluated; the cross-coset step derives coset 7 from the degree
// bound (CrossMap::derive7).  Same polynomial for a trace that satisfies the AIR; for one that does not, the
// out-of-domain identity check (check_ood_identity) reports it instead of the top-block flag.
static int composition_stage(zk_prover *p, Plan *pl, int KX, int C, fe *comp, fe *ctmp, fe *clde, uint8_t root[32],
                             const AirConsts *bnd = nullptr, int nce = 8) {
    const size_t n = (size_t)1 << pl->log_n, CE = 8 * n;
    const int CK = C * KX;
    if (nce != 8 && (nce != 7 || C > 7)) ZK_FAIL(ZK_ERR_INVALID_ARG, "composition: unsupported CE coset count");
    if (nce == 8) ntt(p->st, pl->Tn, comp, n, ctmp, n, 8 * KX, true, nullptr, nullptr, p->tmp);
    else
        for (int j = 0; j < KX; j++) ntt(p->st, pl->Tn, comp + j * CE, n, ctmp + j * CE, n, nce, true, nullptr, nullptr, p->tmp);
    ZK_CHECK_HIP(hipMemsetAsync(p->flag, 0, 4, p->st));
    const fe w8 = h_root_of_unity(3);
    for (int j = 0; j < KX; j++) {
        CrossMap m;
        for (int r = 0; r < 8; r++) m.c[r] = ctmp + (size_t)(8 * j + r) * n;
        m.k0 = 0;
        m.kcount = n;
        m.pstride = (size_t)KX * n;
        if (nce == 7) {
            m.derive7 = 1;
            fe w = w8;
            for (int r = 0; r < 7; r++, w = fe_mul(w, w8)) m.k7[r] = fe_sub(fe_zero(), w);  // -w_8^(r+1)
        }
        comp_cross_mapped(p->st, m, pl->Tce, pl->inv3, h_inv(fe_make(CE)), h_inv(w8), h_inv(h_pow(fe_make(3), n)), C,
                          p->cpolys + (size_t)j * n, p->flag);
    }
    if (bnd)
        for (int j = 0; j < KX; j++)
            boundary_poly_add(p->st, p->polys, pl->log_n, bnd[j], bnd[0].g_last2, p->dscratch, p->cpolys + (size_t)j * n,
                              p->flag);
    return lde_commit(p, pl, p->cpolys, CK, clde, p->cleaves, p->cnodes, root);
}

// Degree check of the composition: the verifier's out-of-domain identity (zk::ood_identity) on the
// frame the proof will carry.  For a trace that satisfies ProcessorAir the composition columns are
// exactly C(x)/Z(x) + boundary quotients, so the identity holds; for any other trace the committed
// columns interpolate a function that is not a polynomial of degree < C*n and the identity fails at the
// transcript-derived z except with probability ~ (degree / p) ~ 2^-100 (Schwartz-Zippel).
// K: the composition coefficients (planes a, b for FieldExtension::Quadratic).
static int check_ood_identity(const std::vector<fe2> &e, int C, const AirConsts *K, int KX, fe2 z, size_t n,
                              const zk_pub_inputs *pub) {
    fe2 ct[NUM_TCONS], cb[NUM_ASSERTS];
    for (int k = 0; k < NUM_TCONS; k++) ct[k] = fe2{K[0].coeff_t[k], KX == 2 ? K[1].coeff_t[k] : fe_zero()};
    for (int k = 0; k < NUM_ASSERTS; k++) cb[k] = fe2{K[0].coeff_b[k], KX == 2 ? K[1].coeff_b[k] : fe_zero()};
    if (!ood_identity(e.data(), C, ct, cb, z, n, pub))
        ZK_FAIL(ZK_ERR_DEGREE, "the trace does not satisfy ProcessorAir (out-of-domain constraint identity failed)");
    return ZK_OK;
}

static int prove_once(zk_prover *p, const TraceSrc &src, size_t n, const zk_options *opt, const zk_pub_inputs *pub,
                      uint8_t *proof_out, size_t *proof_len, zk_record *rec, const zk_dump *dump);

// One proof, plus the hints' bookkeeping for host-resident traces: a hinted sparse column that the host check finds
// nonzero voids the proof, which is redone without hints; a completed proof leaves the columns it found sparse and
// narrow (8- or 32-bit before the last row) as the next proof's hints.
static int prove_impl(zk_prover *p, const TraceSrc &src_in, size_t n, const zk_options *opt, const zk_pub_inputs *pub,
                      uint8_t *proof_out, size_t *proof_len, zk_record *rec, const zk_dump *dump) {
    TraceSrc src = src_in;
    if (dump) src.no_virtual = true;  // the stage dumps read every trace LDE column
    if (src.cols && pub) src.key = &pub->program_hash[0][0];  // hints are per (n, program)
    p->sp_used = false;
    p->sp_hinted = 0;
    p->sp_bad = 0;
    p->clk_used = p->clk_bad = false;
    const size_t cap = proof_len ? *proof_len : 0;  // (in/out: a voided attempt has overwritten it with its length)
    int rc = prove_once(p, src, n, opt, pub, proof_out, proof_len, rec, dump);
    if (!src.cols || !p->sp_used) return rc;
    if (p->sp_bad || p->clk_bad) {
        // a hint of this (n, program) was refuted: forget its column classes (and stop speculating the clock for it if
        // that was refuted), prove again from every column
        zk_prover::HintSet *h = hint_find(p, n, src.key);
        if (h) {
            if (p->clk_bad) h->clk_off = true;
            h->have = false;
            h->sparse = h->nw8 = h->nw32 = 0;
        }
        p->hint_redos++;
        p->clk_used = p->clk_bad = false;
        TraceSrc s2 = src;
        s2.hint_ok = false;
        p->sp_used = false;
        p->sp_bad = 0;
        *proof_len = cap;
        rc = prove_once(p, s2, n, opt, pub, proof_out, proof_len, rec, dump);
        if (!p->sp_used) return rc;
    }
    if (rc == ZK_OK || rc == ZK_ERR_DEGREE || rc == ZK_ERR_BUFFER_TOO_SMALL) {
        // (the hinted sparse columns were not detected on the device: their flags stayed 0, and the host checked them)
        uint32_t found = 0, w8 = 0, w32 = 0;
        for (int c = 0; c < W; c++) {
            if (p->sp_h[c] == 0) found |= 1u << c;
            else if (p->sp_h[W + c] == 0) w8 |= 1u << c;
            else if (p->sp_h[2 * W + c] == 0) w32 |= 1u << c;
        }
        if (p->clk_used) {  // (its flags were not detected on the device) the clock stays in the 32-bit class
            found &= ~1u;
            w8 &= ~1u;
            w32 |= 1u;
        }
        if (src.key) {
            zk_prover::HintSet *h = hint_slot(p, n, src.key);
            h->have = true;
            h->sparse = found;
            h->nw8 = w8;
            h->nw32 = w32;
            h->used = ++p->hint_stamp;
        }
    }
    return rc;
}

static int prove_once(zk_prover *p, const TraceSrc &src, size_t n, const zk_options *opt, const zk_pub_inputs *pub,
                      uint8_t *proof_out, size_t *proof_len, zk_record *rec, const zk_dump *dump) {
    if (!p || !proof_len) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    ZK_REQUIRE_FULL_PROVER(p);
    ZK_TRY(check_prove_args(n, p->max_n, p->max_b, opt, pub));
    // copies from the caller's host columns may still be in flight on an early error return: the caller
    // may free those columns as soon as this returns (a completed proof has long finished them).  Kernels of
    // a failed proof may also still be queued on st: the next proof's uploads into d_trace (on the upload stream,
    // ordered only by the previous proof having drained st) must not race them, so both drain here.
    // proofs in flight on the device: alone, the trace goes up on the latency schedule (trace_lde_commit).  Declared
    // before the copy guard, so this proof counts as in flight until its uploads and kernels have drained.
    DeviceBusy busy{p->dev_busy};
    struct CopyGuard {
        zk_prover *p;
        ~CopyGuard() {
            upload_drain(p);
            (void)hipStreamSynchronize(p->st);
        }
    } copy_guard{p};
    // the AUTO rule (include/zkvm_gpu.h, zk_proof_info): the latency schedule iff no other proof is in flight here
    const int sched = p->upload_sched;
    p->lat_sched = sched == ZK_SCHED_LATENCY || (sched == ZK_SCHED_AUTO && busy.others == 0);
    p->last_sched = src.cols ? (p->lat_sched ? ZK_SCHED_LATENCY : ZK_SCHED_THROUGHPUT) : 0;
    const uint32_t B = opt->blowup, fold = opt->fri_folding;
    const size_t N = n * B;
    ZK_CHECK_HIP(hipSetDevice(p->device));
    IoScope io_scope(p);
    Plan *pl = nullptr;
    ZK_TRY(get_plan(p, n, B, &pl));
    const int log_n = pl->log_n, log_b = pl->log_b;
    const int C = num_comp_cols(n);
    if (C > 8) ZK_FAIL(ZK_ERR_INVALID_ARG, "composition column count exceeds 8");
    const fe g = h_root_of_unity(log_n);
    zk_record R;
    memset(&R, 0, sizeof R);
    R.trace_len = (uint32_t)n;
    R.lde_len = (uint32_t)N;
    R.width = W;
    R.num_ccols = (uint32_t)C;
    stage_begin(p);
    stage_mark(p, "start");

    // S0: coin seed [P1]
    Coin coin = seed_coin(n, opt, pub);

    // S2: trace LDE + commitment
    ZK_TRY(trace_lde_commit(p, pl, src, n, R.trace_root));
    ZK_TRY(d2h_flush(p));
    stage_mark(p, "trace_commit");
    HostTimer HT;
    HT.start();
    coin.reseed(R.trace_root);

    // S3: constraint composition coefficients [P4] and evaluation over the CE domain.  With
    // FieldExtension::Quadratic the coefficients are E values and the composition has two planes
    // (a, b): the evaluator runs once per plane with that component of every coefficient.
    const int KX = (int)opt->field_extension, CK = C * KX;
    if (KX == 2) ZK_TRY(ensure_ext(p));
    fe *comp = KX == 2 ? p->x_comp : p->comp, *ctmp = KX == 2 ? p->x_ctmp : p->ctmp;
    fe *clde = KX == 2 ? p->x_clde : p->clde, *deep = KX == 2 ? p->x_deep : p->deep;
    fe *fri = KX == 2 ? p->x_fri : p->fri;
    // The assertion terms are not evaluated per row here: S4 adds them in coefficient form (unless the
    // caller dumps the composition values, which must then include them).
    const bool bnd_rows = dump && dump->composition;
    // CE cosets evaluated: 7 when the composition has at most 7 columns (the stage derives the 8th)
    const int nce = (!bnd_rows && C <= 7) ? 7 : 8;
    AirConsts Kp[2];
    if (KX == 1) {
        draw_air_consts(coin, pub, n, Kp[0], R);
        ZK_TRY(h2d_small(p, p->air_consts, &Kp[0], sizeof Kp[0]));
        const fe *binv = boundary_inverses(p, pl);
        if (!binv) ZK_FAIL(ZK_ERR_OUT_OF_MEMORY, "boundary divisor table");
        ZK_CHECK_HIP(eval_constraints(p->st, p->lde, log_n, log_b, pl->periodic, binv, (const AirConsts *)p->air_consts, comp,
                                      bnd_rows, nce));
        HT.stop("air_consts");
    } else {
        draw_air_consts_ext(coin, pub, n, Kp[0], Kp[1], R);
        ZK_TRY(h2d_small(p, p->x_air, Kp, sizeof Kp));
        const fe *binv = boundary_inverses(p, pl);
        if (!binv) ZK_FAIL(ZK_ERR_OUT_OF_MEMORY, "boundary divisor table");
        ZK_CHECK_HIP(eval_constraints_ext(p->st, p->lde, log_n, log_b, pl->periodic, binv, (const AirConsts *)p->x_air, comp,
                                          bnd_rows, nce));
    }
    stage_mark(p, "constraints");

    // S4: composition polynomial (interpolate over the CE coset, segment into C columns) + commit.
    ZK_TRY(composition_stage(p, pl, KX, C, comp, ctmp, clde, R.constraint_root, bnd_rows ? nullptr : Kp, nce));
    unsigned degree_flag = 0;
    ZK_TRY(d2h_small(p, &degree_flag, p->flag, 4));
    ZK_TRY(d2h_flush(p));
    stage_mark(p, "composition");
    HT.start();
    coin.reseed(R.constraint_root);

    // FRI layer 0 is the DEEP LDE, coset-major as the coset NTT wrote it (FriLayout lb0 = log_b), unless it is
    // already the remainder (no fold layers), which the host reads in natural order
    const int nl = fri_num_layers(N, opt);
    const int lb0 = nl > 0 ? log_b : 0;
    // S5: OOD frame [P7], DEEP coefficients [P8] and evaluations.  h holds the frame flattened
    // (k base elements per E value): [T(z)]_W ++ [T(zg)]_W ++ [H(z)]_C.
    std::vector<fe> h((2 * W + C) * KX);
    if (KX == 1) {
        const fe z = coin.draw(), zg = fe_mul(z, g);
        fe_to_bytes(z, R.z);
        ood_eval(p->st, p->polys, W, p->cpolys, C, log_n, z, zg, p->ood_tab, p->partials, p->ood);
        HT.stop("z");
        ZK_TRY(d2h_small(p, h.data(), p->ood, (2 * W + C) * sizeof(fe)));
        ZK_TRY(d2h_flush(p));
        HT.start();
        ood_reseed(coin, h.data(), C, R);
        stage_mark(p, "ood");
        const DeepConsts D = draw_deep_consts(coin, h.data(), C, z, zg, R);
        ZK_TRY(h2d_small(p, p->deep_consts, &D, sizeof D));
        deep_coeff_launch(p->st, pl->Tn, p->polys, p->cpolys, C, log_n, log_b, p->deep_consts, z, zg, pl->ct,
                          p->dscratch, p->ulde, p->tmp, lb0 ? nullptr : deep);
        HT.stop("deep_consts");
        // while the GPU runs DEEP: the verifier's out-of-domain identity on the frame just read
        std::vector<fe2> e(2 * W + C);
        for (int i = 0; i < 2 * W + C; i++) e[i] = fe2_lift(h[i]);
        ZK_TRY(check_ood_identity(e, C, Kp, 1, fe2_lift(z), n, pub));
    } else {
        const fe2 z = coin.draw_ext(2), zg = fe2_mulb(z, g);
        fe_to_bytes(z.a, R.z);
        const int np = 2 * W + CK;  // E values of the trace polys at z, zg and of the C*k base composition polys at z
        ood_eval_ext(p->st, p->polys, W, p->cpolys, CK, log_n, z, zg, p->x_tab, p->x_partials, p->ood);
        std::vector<fe> hv(2 * np);
        ZK_TRY(d2h_small(p, hv.data(), p->ood, hv.size() * sizeof(fe)));
        ZK_TRY(d2h_flush(p));
        std::vector<fe2> e;
        ood_reseed_ext(coin, hv, C, R, e, h);
        stage_mark(p, "ood");
        const DeepConstsE D = draw_deep_consts_ext(coin, e, C, z, zg, R);
        ZK_TRY(h2d_small(p, p->x_deep_consts, &D, sizeof D));
        deep_coeff_ext_launch(p->st, pl->Tn, p->polys, p->cpolys, C, log_n, log_b, p->x_deep_consts, z, zg,
                              pl->ct, p->x_dscratch, p->x_ulde, p->tmp, lb0 ? nullptr : deep);
        ZK_TRY(check_ood_identity(e, C, Kp, 2, z, n, pub));
    }
    stage_mark(p, "deep");

    // S6: FRI [P9, P10]; E layers are planar (k planes of L values)
    if (nl > ZK_MAX_FRI_LAYERS) ZK_FAIL(ZK_ERR_INVALID_ARG, "too many FRI layers");
    R.num_fri_layers = (uint32_t)nl;
    {
        size_t tot = 0, s = N;
        for (int l = 0; l < nl; l++) tot += (s /= fold);
        if (tot > p->max_n * p->max_b) ZK_FAIL(ZK_ERR_INVALID_ARG, "FRI layers exceed the prover's buffers");
    }
    std::vector<const fe *> layer_vals(nl + 1);
    std::vector<uint8_t *> layer_leaves(nl), layer_nodes(nl);
    std::vector<size_t> layer_len(nl + 1);
    std::vector<fe> rem_flat;
    const fe *deep0 = lb0 ? (KX == 2 ? p->x_ulde : p->ulde) : deep;
    layer_vals[0] = deep0;
    layer_len[0] = N;
    {
        // The layer coins run on the device (fri_coin_launch): no host round trip per layer.  The
        // constant part of the fold constants is uploaded once; each layer's coin writes alpha into it.
        fe *next = fri;
        uint8_t *dig = p->fri_dig;
        fe *alpha_dev = nullptr;
        if (KX == 1) {
            const FoldConsts F = fold_consts(fe_zero(), fold);
            ZK_TRY(h2d_small(p, p->fold_consts, &F, sizeof F));
            alpha_dev = &((FoldConsts *)p->fold_consts)->alpha;
        } else {
            const FoldConstsE F = fold_consts_ext(fe2_zero(), fold);
            ZK_TRY(h2d_small(p, p->x_fold_consts, &F, sizeof F));
            alpha_dev = &((FoldConstsE *)p->x_fold_consts)->alpha.a;
        }
        ZK_TRY(h2d_small(p, p->fri_seed, coin.seed, 32));
        for (int l = 0; l < nl; l++) {
            const size_t L = layer_len[l], rows = L / fold;
            layer_leaves[l] = dig;
            layer_nodes[l] = dig + 32 * rows;
            dig += 64 * rows;
            const int lb = l ? 0 : lb0;
            if (KX == 1) commit_fri_layer(p->st, layer_vals[l], L, (int)fold, layer_leaves[l], layer_nodes[l], lb);
            else commit_fri_layer_ext(p->st, layer_vals[l], L, (int)fold, layer_leaves[l], layer_nodes[l], lb);
            fri_coin_launch(p->st, (uint32_t *)p->fri_seed, layer_nodes[l] + 32, KX, alpha_dev, p->fri_alphas + 2 * l);
            if (KX == 1) fri_fold_launch(p->st, layer_vals[l], L, (int)fold, p->fold_consts, pl->TN, N / L, next, lb);
            else fri_fold_ext_launch(p->st, layer_vals[l], L, (int)fold, p->x_fold_consts, pl->TN, N / L, next, lb);
            layer_vals[l + 1] = next;
            layer_len[l + 1] = rows;
            next += KX * rows;
        }
        // one round trip for the whole commit phase: roots, device alphas, the last layer
        const size_t L = layer_len[nl];
        std::vector<fe> rv(KX * L), dalpha(2 * nl);
        for (int l = 0; l < nl; l++) ZK_TRY(d2h_small(p, R.fri_roots[l], layer_nodes[l] + 32, 32));
        if (nl) ZK_TRY(d2h_small(p, dalpha.data(), p->fri_alphas, 2 * nl * sizeof(fe)));
        ZK_TRY(d2h_small(p, rv.data(), layer_vals[nl], rv.size() * sizeof(fe)));
        ZK_TRY(d2h_flush(p));
        HT.start();
        // host replay of the same transcript (it continues into the remainder, grinding and queries)
        for (int l = 0; l < nl; l++) {
            coin.reseed(R.fri_roots[l]);
            const fe2 alpha = KX == 1 ? fe2{coin.draw(), fe_zero()} : coin.draw_ext(2);
            fe_to_bytes(alpha.a, R.fri_alphas[l]);
            if (!fe_eq(alpha.a, dalpha[2 * l]) || (KX == 2 && !fe_eq(alpha.b, dalpha[2 * l + 1])))
                ZK_FAIL(ZK_ERR_DEVICE, "device FRI transcript diverged from the host transcript");
        }
        HT.stop("fri_replay");
        HT.start();
        if (KX == 1) ZK_TRY(remainder_step(rv, B, coin, R, degree_flag));
        else ZK_TRY(remainder_step_ext(rv, B, coin, R, degree_flag, rem_flat));
    }
    stage_mark(p, "fri");

    HT.stop("remainder");
    HT.start();
    // S7: grinding and query positions [P10, P11]
    std::vector<uint64_t> pos;
    ZK_TRY(grind_and_positions(p, coin, opt, N, R, pos));
    const size_t nu = pos.size();
    const auto fri_pos = fri_fold_positions(pos, N, fold, nl);
    HT.stop("positions");
    HT.start();

    // S8: openings.  Every value and digest the proof opens, as a list of 16-byte device chunks: one
    // address upload, one gather kernel, one download.
    // The Openings and the address list live in the prover (pinned / capacity kept across proofs):
    // fresh host allocations here cost page faults on every proof (~100 us at 2^20).
    if (!p->open) p->open = new Openings();
    Openings &O = *p->open;
    O.reset(2 + nl);
    plan_batch(N, pos, O.plans[0]);
    O.plans[1] = O.plans[0];  // the composition tree opens the same positions
    for (int l = 0; l < nl; l++) plan_batch(layer_len[l] / fold, fri_pos[l], O.plans[2 + l]);
    uint64_t *addr = p->h_gather_idx;
    size_t na = 0;
    auto fe_at = [&](const fe *base, size_t idx) { addr[na++] = (uint64_t)(uintptr_t)(base + idx); };
    auto row_at = [&](const fe *base, int ncols, uint64_t i) {  // coset-major LDE row i
        for (int c = 0; c < ncols; c++) {
            if (base == p->lde && ((p->virt >> c) & 1u)) fe_at(p->virt_lagr, (i & (B - 1)) * n + (i >> log_b));
            else fe_at(base, ((size_t)c * B + (i & (B - 1))) * n + (i >> log_b));
        }
    };
    size_t need = nu * (W + CK);
    for (int l = 0; l < nl; l++) need += fri_pos[l].size() * fold * KX;
    for (int b = 0; b < 2 + nl; b++) need += 2 * O.plans[b].count();
    if (need > ZK_GATHER_CAP) ZK_FAIL(ZK_ERR_INVALID_ARG, "too many opened values for the gather buffer");
    for (size_t q = 0; q < nu; q++) row_at(p->lde, W, pos[q]);
    for (size_t q = 0; q < nu; q++) row_at(clde, CK, pos[q]);
    for (int l = 0; l < nl; l++) {
        const size_t rows = layer_len[l] / fold;
        for (uint64_t r : fri_pos[l])
            for (uint32_t k = 0; k < fold; k++)
                for (int j = 0; j < KX; j++) {
                    const uint64_t i = r + k * rows;  // natural index in layer l
                    fe_at(layer_vals[l], j * layer_len[l] + ((l || !lb0) ? i : ((i & (B - 1)) << log_n) + (i >> log_b)));
                }
    }
    const size_t off_dig = na;
    for (int b = 0; b < 2 + nl; b++) {
        const uint8_t *lv = b == 0 ? p->leaves : b == 1 ? p->cleaves : layer_leaves[b - 2];
        const uint8_t *nd = b == 0 ? p->nodes : b == 1 ? p->cnodes : layer_nodes[b - 2];
        for (auto &path : O.plans[b].paths)
            for (auto &e : path) {
                const uint8_t *d = (e.first ? nd : lv) + 32 * e.second;
                addr[na++] = (uint64_t)(uintptr_t)d;
                addr[na++] = (uint64_t)(uintptr_t)(d + 16);
            }
    }
    HT.stop("plans_addresses");
    ZK_CHECK_HIP(hipMemcpyAsync(p->gather_idx, p->h_gather_idx, na * 8, hipMemcpyHostToDevice, p->st));
    gather_chunks(p->st, p->gather_idx, na, p->gather_out);
    ZK_CHECK_HIP(hipMemcpyAsync(p->h_gather_out, p->gather_out, na * sizeof(fe), hipMemcpyDeviceToHost, p->st));
    ZK_CHECK_HIP(hipStreamSynchronize(p->st));
    {
        const fe *got = p->h_gather_out;
        size_t off = 0;
        O.trace_rows.assign(got, got + nu * W);
        if (p->virt)  // virtual columns: the gather read e_(n-1)'s LDE there; times the column's last row
            for (size_t q = 0; q < nu; q++)
                for (int c = 0; c < W; c++)
                    if ((p->virt >> c) & 1u) O.trace_rows[q * W + c] = fe_mul(O.trace_rows[q * W + c], p->virt_last[c]);
        off += nu * W;
        O.comp_rows.assign(got + off, got + off + nu * CK);
        off += nu * CK;
        for (int l = 0; l < nl; l++) {
            O.fri_rows[l].assign(got + off, got + off + fri_pos[l].size() * fold * KX);
            off += fri_pos[l].size() * fold * KX;
        }
        const uint8_t *dg = (const uint8_t *)(got + off_dig);
        for (int b = 0; b < 2 + nl; b++) {
            const size_t bytes = 32 * O.plans[b].count();
            O.digests[b].assign(dg, dg + bytes);
            dg += bytes;
        }
    }
    stage_mark(p, "queries");

    // S9: proof bytes [P13, P14]
    HT.start();
    std::vector<uint8_t> &bytes = p->proof_bytes;
    serialize_proof(n, opt, C, R, h.data(), O, KX == 2 ? &rem_flat : nullptr, bytes);
    HT.stop("serialize");
    stage_mark(p, "serialize");
    ZK_CHECK_HIP(hipStreamSynchronize(p->st));
    stage_collect(p);
    collect_kernel_stats(p);

    if (rec) *rec = R;
    if (dump) {  // E-valued stages dump their a component (as the oracle does)
        if (dump->trace_polys) ZK_CHECK_HIP(hipMemcpy(dump->trace_polys, p->polys, (size_t)W * n * 16, hipMemcpyDeviceToHost));
        if (dump->trace_lde) coset_major_rows_to_host(p, p->lde, W, n, B, dump->trace_lde);
        if (dump->trace_leaves) ZK_CHECK_HIP(hipMemcpy(dump->trace_leaves, p->leaves, 32 * N, hipMemcpyDeviceToHost));
        if (dump->composition) coset_major_rows_to_host(p, comp, 1, n, 8, dump->composition);
        if (dump->comp_polys) ZK_CHECK_HIP(hipMemcpy(dump->comp_polys, p->cpolys, (size_t)CK * n * 16, hipMemcpyDeviceToHost));
        if (dump->comp_lde) coset_major_rows_to_host(p, clde, CK, n, B, dump->comp_lde);
        if (dump->deep) {
            if (lb0) coset_major_to_natural(p->st, deep0, log_n, log_b, deep);
            ZK_CHECK_HIP(hipStreamSynchronize(p->st));
            ZK_CHECK_HIP(hipMemcpy(dump->deep, deep, N * 16, hipMemcpyDeviceToHost));
        }
        if (dump->fri_layer1 && nl > 0)
            ZK_CHECK_HIP(hipMemcpy(dump->fri_layer1, layer_vals[1], layer_len[1] * 16, hipMemcpyDeviceToHost));
    }
    p->last_n = n;
    p->last_b = B;
    return deliver_proof(bytes, degree_flag, proof_out, proof_len);
}

int zk_prove_device(zk_prover *p, const void *d_trace, size_t n, const zk_options *opt, const zk_pub_inputs *pub,
                    uint8_t *proof_out, size_t *proof_len, zk_record *rec, const zk_dump *dump) {
    if (!d_trace) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    TraceSrc src;
    src.dev = (const fe *)d_trace;
    return prove_impl(p, src, n, opt, pub, proof_out, proof_len, rec, dump);
}

int zk::fixed_prefix(zk_prover *p, size_t n, uint32_t B, const FixedCols &fx) {
    p->fix_prefix_blocks = 0;
    Plan *pl = nullptr;
    ZK_TRY(get_plan(p, n, B, &pl));
    if (!p->fix_ws) ZK_CHECK_HIP(p->arena.alloc(&p->fix_ws, W));
    fe_ws ws[W];
    for (int c = 0; c < W; c++) ws[c] = make_fe_ws(fx.last[c]);
    ZK_TRY(h2d_small(p, p->fix_ws, ws, sizeof ws));
    fixed_axpy(p->st, fx, p->fix_ws, n, (size_t)1 << pl->log_b, p->polys, p->lde);
    constexpr int nb = 12 / 4;  // columns 0 .. 11 are preprocessed whatever the program's stack depth
    hash_rows_blocks(p->st, p->lde, W, pl->log_n, pl->log_b, 0, nb, p->leaves);
    p->fix_prefix_blocks = nb;
    return ZK_OK;
}

int zk::prove_fixed(zk_prover *p, size_t n, const zk_options *opt, const zk_pub_inputs *pub, const FixedCols *fx,
                    uint8_t *proof_out, size_t *proof_len) {
    TraceSrc src;
    src.dev = p->d_trace;
    src.fixed = fx;
    return prove_impl(p, src, n, opt, pub, proof_out, proof_len, nullptr, nullptr);
}

int zk::prove_single(zk_prover *p, const uint8_t *trace, size_t n, const zk_options *opt, const zk_pub_inputs *pub,
                     uint8_t *proof_out, size_t *proof_len, zk_record *rec) {
    const uint8_t *cols[W];
    TraceSrc src;
    if (trace) {
        for (int c = 0; c < W; c++) cols[c] = trace + (size_t)c * n * sizeof(fe);
        src.cols = cols;
    } else {
        src.dev = p->d_trace;
    }
    return prove_impl(p, src, n, opt, pub, proof_out, proof_len, rec, nullptr);
}

int zk_prove_columns_ex(zk_prover *p, const uint8_t *const *columns, size_t n, const zk_options *opt,
                        const zk_pub_inputs *pub, uint8_t *proof_out, size_t *proof_len, zk_record *rec,
                        const zk_dump *dump) {
    if (!columns) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    for (int c = 0; c < W; c++)
        if (!columns[c]) ZK_FAIL(ZK_ERR_INVALID_ARG, "null trace column");
    TraceSrc src;
    src.cols = columns;
    return prove_impl(p, src, n, opt, pub, proof_out, proof_len, rec, dump);
}

int zk_prove_columns(zk_prover *p, const uint8_t *const *columns, size_t n, const zk_options *opt,
                     const zk_pub_inputs *pub, uint8_t *proof_out, size_t *proof_len) {
    return zk_prove_columns_ex(p, columns, n, opt, pub, proof_out, proof_len, nullptr, nullptr);
}

int zk_prove(zk_prover *p, const uint8_t *trace, size_t n, const zk_options *opt, const zk_pub_inputs *pub,
             uint8_t *proof_out, size_t *proof_len) {
    if (!trace) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    const uint8_t *cols[W];
    for (int c = 0; c < W; c++) cols[c] = trace + (size_t)c * n * sizeof(fe);
    return zk_prove_columns(p, cols, n, opt, pub, proof_out, proof_len);
}

// ---------------------------------------------------------------- page-locked host memory for traces
int zk_host_alloc(size_t bytes, void **ptr) {
    if (!ptr || !bytes) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    *ptr = nullptr;
    const hipError_t e = hipHostMalloc(ptr, bytes, hipHostMallocPortable);
    if (e != hipSuccess) {
        *ptr = nullptr;
        ZK_CHECK_HIP(e);
    }
    return ZK_OK;
}

void zk_host_free(void *ptr) {
    if (ptr) (void)hipHostFree(ptr);
}

int zk_host_register(void *ptr, size_t bytes) {
    if (!ptr || !bytes) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    ZK_CHECK_HIP(hipHostRegister(ptr, bytes, hipHostRegisterPortable));
    return ZK_OK;
}

int zk_host_unregister(void *ptr) {
    if (!ptr) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    ZK_CHECK_HIP(hipHostUnregister(ptr));
    return ZK_OK;
}

// ---------------------------------------------------------------- plug point 1: trace LDE
int zk_lde_new(zk_prover *p, const uint8_t *trace, size_t width, size_t n, uint32_t blowup, zk_trace_lde **out,
               uint8_t root[32]) {
    if (!p || !trace || !out) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    ZK_REQUIRE_FULL_PROVER(p);
    if (width != (size_t)W) ZK_FAIL(ZK_ERR_INVALID_ARG, "ProcessorAir traces have 28 columns");
    if (n < 16 || (n & (n - 1)) || n > p->max_n || blowup < 8 || (blowup & (blowup - 1)) || blowup > p->max_b)
        ZK_FAIL(ZK_ERR_INVALID_ARG, "invalid trace length or blowup");
    ZK_CHECK_HIP(hipSetDevice(p->device));
    IoScope io_scope(p);
    Plan *pl;
    int rc = get_plan(p, n, blowup, &pl);
    if (rc) return rc;
    const uint8_t *cols[W];
    for (int c = 0; c < W; c++) cols[c] = trace + (size_t)c * n * sizeof(fe);
    TraceSrc src;
    src.cols = cols;
    src.hint_ok = false;  // no proof follows to verify a hint
    uint8_t r[32];
    rc = trace_lde_commit(p, pl, src, n, r);
    if (!rc) rc = d2h_flush(p);
    upload_drain(p);  // the caller's trace is no longer read once this returns
    if (rc) return rc;
    if (root) memcpy(root, r, 32);
    *out = new zk_trace_lde{p, n, blowup, W};
    return ZK_OK;
}

int zk_lde_read_frame(zk_trace_lde *h, size_t step, uint8_t *cur, uint8_t *next) {
    if (!h || !cur || !next) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    zk_prover *p = h->p;
    const size_t N = h->n * h->B;
    if (step >= N) ZK_FAIL(ZK_ERR_INVALID_ARG, "lde_step out of range");
    uint64_t idx[2] = {step, (step + h->B) % N};
    ZK_CHECK_HIP(hipMemcpyAsync(p->gather_idx, idx, 16, hipMemcpyHostToDevice, p->st));
    gather_rows(p->st, p->lde, W, ilog2(h->n), ilog2(h->B), p->gather_idx, 2, p->gather_out);
    fe rows[2 * W];
    ZK_CHECK_HIP(hipMemcpyAsync(rows, p->gather_out, sizeof rows, hipMemcpyDeviceToHost, p->st));
    ZK_CHECK_HIP(hipStreamSynchronize(p->st));
    memcpy(cur, rows, W * 16);
    memcpy(next, rows + W, W * 16);
    return ZK_OK;
}

// rows at `positions` of a committed coset-major LDE (ncols columns) + the batch Merkle proof bytes
static int query_committed_rows(zk_prover *p, const fe *base, int ncols, size_t n, uint32_t B, const uint8_t *leaves,
                                const uint8_t *nodes, const uint64_t *positions, size_t k, uint8_t *rows_out,
                                uint8_t *proof_out, size_t *proof_len) {
    if (!positions || !rows_out || !proof_len || k == 0 || k > ZK_MAX_QUERIES)
        ZK_FAIL(ZK_ERR_INVALID_ARG, "invalid query arguments");
    const size_t N = n * B;
    std::vector<uint64_t> pos(positions, positions + k);
    for (uint64_t x : pos)
        if (x >= N) ZK_FAIL(ZK_ERR_INVALID_ARG, "query position out of range");
    ZK_CHECK_HIP(hipMemcpyAsync(p->gather_idx, pos.data(), k * 8, hipMemcpyHostToDevice, p->st));
    gather_rows(p->st, base, ncols, ilog2(n), ilog2(B), p->gather_idx, k, p->gather_out);
    ZK_CHECK_HIP(hipMemcpyAsync(rows_out, p->gather_out, k * ncols * 16, hipMemcpyDeviceToHost, p->st));
    ZK_CHECK_HIP(hipStreamSynchronize(p->st));
    BatchPlan bp = plan_batch(N, pos);
    Bytes out;
    out.u8((uint8_t)bp.paths.size());
    for (auto &path : bp.paths) {
        out.u8((uint8_t)path.size());
        for (auto &e : path) {
            uint8_t d[32];
            ZK_CHECK_HIP(hipMemcpy(d, (e.first ? nodes : leaves) + 32 * e.second, 32, hipMemcpyDeviceToHost));
            out.put(d, 32);
        }
    }
    size_t cap = *proof_len;
    *proof_len = out.v.size();
    if (!proof_out || cap < out.v.size()) ZK_FAIL(ZK_ERR_BUFFER_TOO_SMALL, "proof buffer too small");
    memcpy(proof_out, out.v.data(), out.v.size());
    return ZK_OK;
}

int zk_lde_query(zk_trace_lde *h, const uint64_t *positions, size_t k, uint8_t *rows_out, uint8_t *proof_out,
                 size_t *proof_len) {
    if (!h) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    zk_prover *p = h->p;
    return query_committed_rows(p, p->lde, W, h->n, h->B, p->leaves, p->nodes, positions, k, rows_out, proof_out,
                                proof_len);
}

void zk_lde_free(zk_trace_lde *h) { delete h; }

// ---------------------------------------------------------------- plug point 2: constraint evaluation
int zk_eval_constraints(zk_trace_lde *h, const zk_pub_inputs *pub, const uint8_t *coeff_t, const uint8_t *coeff_b,
                        uint8_t *out) {
    if (!h || !pub || !coeff_t || !coeff_b || !out) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    if (pub->lwe_size == 0 || pub->lwe_size > 5) ZK_FAIL(ZK_ERR_INVALID_ARG, "lwe_size must be in [1, 5]");
    zk_prover *p = h->p;
    const size_t n = h->n;
    Plan *pl;
    int rc = get_plan(p, n, h->B, &pl);
    if (rc) return rc;
    AirConsts K;
    memset(&K, 0, sizeof K);
    for (int k = 0; k < NUM_TCONS; k++) K.coeff_t[k] = fe_from_bytes(coeff_t + 16 * k);
    for (int k = 0; k < NUM_ASSERTS; k++) K.coeff_b[k] = fe_from_bytes(coeff_b + 16 * k);
    air_static_consts(pub, n, K);
    ZK_CHECK_HIP(hipMemcpyAsync(p->air_consts, &K, sizeof K, hipMemcpyHostToDevice, p->st));
    const fe *binv = boundary_inverses(p, pl);
    if (!binv) ZK_FAIL(ZK_ERR_OUT_OF_MEMORY, "boundary divisor table");
    ZK_CHECK_HIP(eval_constraints(p->st, p->lde, pl->log_n, pl->log_b, pl->periodic, binv, (const AirConsts *)p->air_consts,
                                  p->comp));
    ZK_CHECK_HIP(hipStreamSynchronize(p->st));
    coset_major_rows_to_host(p, p->comp, 1, n, 8, out);
    return ZK_OK;
}

// ---------------------------------------------------------------- plug point 3: constraint commitment
struct zk_comp_commit {
    zk_prover *p;
    size_t n;
    uint32_t B;
    int ncols;
};

int zk_commit_composition(zk_trace_lde *h, const uint8_t *composition, uint32_t num_cols, zk_comp_commit **out,
                          uint8_t root[32], uint8_t *polys_out) {
    if (!h || !composition || !out) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    if (num_cols < 1 || num_cols > 8) ZK_FAIL(ZK_ERR_INVALID_ARG, "num_cols must be in [1, 8]");
    zk_prover *p = h->p;
    const size_t n = h->n, CE = 8 * n;
    ZK_CHECK_HIP(hipSetDevice(p->device));
    IoScope io_scope(p);
    Plan *pl;
    int rc = get_plan(p, n, h->B, &pl);
    if (rc) return rc;
    // natural CE order (step i = r + 8q) -> coset-major comp[r*n + q], the evaluator's layout
    std::vector<fe> cm(CE);
    const fe *in = reinterpret_cast<const fe *>(composition);
    for (size_t i = 0; i < CE; i++) memcpy(&cm[(i & 7) * n + (i >> 3)], in + i, sizeof(fe));
    ZK_CHECK_HIP(hipMemcpyAsync(p->comp, cm.data(), CE * sizeof(fe), hipMemcpyHostToDevice, p->st));
    uint8_t r[32];
    if ((rc = composition_stage(p, pl, 1, (int)num_cols, p->comp, p->ctmp, p->clde, r))) return rc;
    unsigned degree_flag = 0;
    if ((rc = d2h_small(p, &degree_flag, p->flag, 4)) || (rc = d2h_flush(p))) return rc;  // root and flag
    if (degree_flag) ZK_FAIL(ZK_ERR_DEGREE, "composition polynomial degree exceeds num_cols * trace_len");
    if (polys_out)
        ZK_CHECK_HIP(hipMemcpy(polys_out, p->cpolys, (size_t)num_cols * n * sizeof(fe), hipMemcpyDeviceToHost));
    if (root) memcpy(root, r, 32);
    *out = new zk_comp_commit{p, n, h->B, (int)num_cols};
    return ZK_OK;
}

int zk_comp_query(zk_comp_commit *h, const uint64_t *positions, size_t k, uint8_t *rows_out, uint8_t *proof_out,
                  size_t *proof_len) {
    if (!h) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    zk_prover *p = h->p;
    return query_committed_rows(p, p->clde, h->ncols, h->n, h->B, p->cleaves, p->cnodes, positions, k, rows_out,
                                proof_out, proof_len);
}

void zk_comp_free(zk_comp_commit *h) { delete h; }

// ---------------------------------------------------------------- diagnostics
// Host execution of the lazy dot product (acc288: unreduced 256-bit products, one reduction)
extern "C" void zk_diag_dot_host(const uint8_t *a, const uint8_t *b, size_t count, uint8_t *out) {
    acc288 acc = acc288_zero();
    for (size_t i = 0; i < count; i++) acc288_madd(acc, fe_from_bytes(a + 16 * i), fe_from_bytes(b + 16 * i));
    fe_to_bytes(acc288_reduce(acc), out);
}

// Host execution of the exact device multiply (fe_mul_limbs) -- lets CPU tests check the GPU
// reduction algorithm without a GPU.
extern "C" void zk_diag_mul_limbs_host(const uint8_t *a, const uint8_t *b, uint8_t *out, size_t count) {
    for (size_t i = 0; i < count; i++) fe_to_bytes(fe_mul_limbs(fe_from_bytes(a + 16 * i), fe_from_bytes(b + 16 * i)), out + 16 * i);
}
extern "C" void zk_diag_blake3_host(const uint8_t *in, size_t len, uint8_t out[32]) { b3::hash_bytes(in, len, out); }

// GPU elementwise field op: 0 add, 1 sub, 2 mul, 3 inv(a), 4 a^b (b as a 128-bit exponent), 5 lazy add,
// 6 canonical form of a, 7 multiply by b in two-part form
extern "C" int zk_diag_field_op(int device, int op, const uint8_t *a, const uint8_t *b, uint8_t *out, size_t count) {
    if (!a || !b || !out || count == 0) ZK_FAIL(ZK_ERR_INVALID_ARG, "null argument");
    ZK_CHECK_HIP(hipSetDevice(device));
    fe *d = nullptr;
    ZK_CHECK_HIP(hipMalloc(&d, 3 * count * sizeof(fe)));
    ZK_CHECK_HIP(hipMemcpy(d, a, count * 16, hipMemcpyHostToDevice));
    ZK_CHECK_HIP(hipMemcpy(d + count, b, count * 16, hipMemcpyHostToDevice));
    diag_field_op(nullptr, op, d, d + count, d + 2 * count, count);
    hipError_t e = hipMemcpy(out, d + 2 * count, count * 16, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    ZK_CHECK_HIP(e);
    return ZK_OK;
}

// GPU BLAKE3 of `count` rows of k field elements (k <= 64)
extern "C" int zk_diag_blake3_rows(int device, const uint8_t *rows, int k, size_t count, uint8_t *out) {
    if (!rows || !out || k <= 0 || k > 64 || count == 0) ZK_FAIL(ZK_ERR_INVALID_ARG, "invalid argument");
    ZK_CHECK_HIP(hipSetDevice(device));
    fe *d = nullptr;
    ZK_CHECK_HIP(hipMalloc(&d, count * k * sizeof(fe) + 32 * count));
    ZK_CHECK_HIP(hipMemcpy(d, rows, count * k * 16, hipMemcpyHostToDevice));
    uint8_t *dout = (uint8_t *)(d + count * k);
    diag_blake3_elems(nullptr, d, k, count, dout);
    hipError_t e = hipMemcpy(out, dout, 32 * count, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    ZK_CHECK_HIP(e);
    return ZK_OK;
}

// GPU NTT of `batch` polys of size n: inverse != 0 -> interpolation (with 1/n), else evaluation
// over offset * <w_n> (offset given as 16 bytes; pass 1 for the plain subgroup)
extern "C" int zk_diag_ntt(int device, const uint8_t *in, size_t n, int batch, int inverse, const uint8_t *offset,
                           uint8_t *out) {
    if (!in || !out || n < 2 || (n & (n - 1)) || batch <= 0) ZK_FAIL(ZK_ERR_INVALID_ARG, "invalid argument");
    zk_prover *p = nullptr;
    int rc = zk_prover_create(device, std::max<size_t>(n, 16), 8, &p);
    if (rc) return rc;
    std::unique_ptr<zk_prover, void (*)(zk_prover *)> guard(p, zk_prover_destroy);
    NttTables T;
    ZK_CHECK_HIP(make_ntt_tables(p, ilog2(n), &T));
    if (T.log_n > 12) {
        ZK_CHECK_HIP(p->arena.alloc(&T.fwd_pass, n));
        ZK_CHECK_HIP(p->arena.alloc(&T.inv_pass, n));
        make_pass_twiddles(p->st, T);
    }
    PowTable pre;
    fe off = offset ? fe_from_bytes(offset) : fe_one();
    bool use_pre = !inverse && !fe_eq(off, fe_one());
    if (use_pre) ZK_CHECK_HIP(make_pow_table(p, off, n, &pre));
    fe *d_in = nullptr, *d_out = nullptr, *d_tmp = nullptr;
    ZK_CHECK_HIP(p->arena.alloc(&d_in, n * batch));
    ZK_CHECK_HIP(p->arena.alloc(&d_out, n * batch));
    ZK_CHECK_HIP(p->arena.alloc(&d_tmp, n * batch));
    ZK_CHECK_HIP(hipMemcpy(d_in, in, n * batch * 16, hipMemcpyHostToDevice));
    fe inv_n = h_inv(fe_make(n));
    ntt(p->st, T, d_in, n, d_out, n, batch, inverse != 0, use_pre ? &pre : nullptr, inverse ? &inv_n : nullptr, d_tmp);
    ZK_CHECK_HIP(hipStreamSynchronize(p->st));
    ZK_CHECK_HIP(hipMemcpy(out, d_out, n * batch * 16, hipMemcpyDeviceToHost));
    return ZK_OK;
}
