// prover_internal.hpp -- host-side state and protocol steps shared by the single-GPU prover
// (prover.hip) and the coset-sharded multi-GPU prover (shard.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <string.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/zkvm_gpu.h"
#include "air_shape.hpp"
#include "host_field.hpp"
#include "zk_internal.hpp"

namespace zk {

extern thread_local std::string g_err;

#define ZK_CHECK_HIP(expr)                                                                     \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) {                                                                \
            ::zk::g_err = std::string("HIP error: ") + hipGetErrorString(e_) + " at " #expr;   \
            return e_ == hipErrorOutOfMemory ? ZK_ERR_OUT_OF_MEMORY : ZK_ERR_DEVICE;           \
        }                                                                                      \
    } while (0)

#define ZK_FAIL(code, msg)    \
    do {                      \
        ::zk::g_err = (msg);  \
        return (code);        \
    } while (0)

#define ZK_TRY(expr)                 \
    do {                             \
        int rc_ = (expr);            \
        if (rc_ != ZK_OK) return rc_; \
    } while (0)

static constexpr int W = ZK_TRACE_WIDTH;
// a host-resident trace is uploaded in up to this many column groups (trace_lde_commit; shard.hip: one per round
// of its column split, ceil(W / G) rounds)
static constexpr int ZK_UPLOAD_GROUPS_MAX = 14;
static constexpr int NUM_TCONS = 20;
static constexpr int NUM_ASSERTS = 22;

// single-GPU entry points refuse a prover sized for one rank of a sharded proof
#define ZK_REQUIRE_FULL_PROVER(p)                                                                                  \
    do {                                                                                                          \
        if ((p)->shard_world > 1)                                                                                 \
            ZK_FAIL(ZK_ERR_INVALID_ARG, "this prover was created for one rank of a sharded proof (zk_prover_create_shard)"); \
    } while (0)

inline int ilog2(size_t n) {
    int r = 0;
    while (((size_t)1 << r) < n) r++;
    return r;
}

// ---------------------------------------------------------------- device state
struct DeviceArena {
    std::vector<void *> ptrs;
    ~DeviceArena() {
        for (void *p : ptrs) (void)hipFree(p);
    }
    template <typename T>
    hipError_t alloc(T **p, size_t count) {
        void *q = nullptr;
        hipError_t e = hipMalloc(&q, count * sizeof(T) + 256);
        if (e == hipSuccess) {
            ptrs.push_back(q);
            *p = (T *)q;
        }
        return e;
    }
};

struct Plan {  // everything that depends only on (n, B)
    int log_n = 0, log_b = 0;
    NttTables Tn, Tce, TN;        // sizes n, 8n, B*n
    std::vector<PowTable> coset;  // (3 * w_N^r)^k, r < B (split tables)
    CosetTables ct;               // coset-LDE tables (zk_internal.hpp)
    fe *xn_N = nullptr;           // (3 * w_N^r)^n, r < B: x^n on LDE coset r
    PowTable inv3;                // 3^-k, k < n
    fe *xr_ce = nullptr, *xr_N = nullptr;  // 3 * w_CE^r (8), 3 * w_N^r (B)
    fe *periodic = nullptr;               // 128 x 9
    // 1 / ((x - 1)(x - g^(n-2))) over the CE domain (coset-major): the two boundary divisors
    // depend only on n, so they are inverted once per plan (first proof) and reused
    fe *bnd_inv = nullptr;
    // ... and the same three planes over a sharded rank's block of cosets sh_divs_r0 .. + sh_divs_cos - 1 (shard.hip S3:
    // built on the rank's first proof of this length, reused by the next)
    fe *sh_divs = nullptr;
    int sh_divs_r0 = -1, sh_divs_cos = 0;
    // four-step plans: the interpolant of e_(n-1) (n coefficients) and its coset LDE (B n, coset-major) -- what a
    // trace column that is zero but in its random last row interpolates and extends to, times that row (SparseCols)
    fe *lagr = nullptr, *lagr_lde = nullptr;
    // ... and the column 0, 1, ..., n-1's (the AIR clock of a valid trace but for its random last row), built on first
    // use (clock_tables)
    fe *id_poly = nullptr, *id_lde = nullptr;
    // the LDE cosets lagr_lde / id_lde hold: slot j is coset lde_r0 + (j << lde_shift), lde_cos of them -- all B for
    // a full prover; a rank-sized prover's own B / G (plan_rank_tables), so its tables are sized like its LDE buffers
    int lde_r0 = 0, lde_shift = 0, lde_cos = 0;
    size_t lde_slot(int r) const { return (size_t)((r - lde_r0) >> lde_shift); }
};
// A rank-sized prover's lagr_lde / id_lde over its rank's block of B / G cosets r0 .. r0 + B / G - 1: built on the first
// sharded proof of the plan, rebuilt if the prover serves another rank
int plan_rank_tables(zk_prover *p, Plan *pl, int r0, int G);
// the plan's cached boundary-divisor inverses, computed on first use (stream-ordered)
// the evaluator's divisor tables for the 8 CE cosets (divisor_tables: 3 planes of 8n), built once per plan
const fe *boundary_inverses(zk_prover *p, Plan *pl);
// 1 / (x^n - 1) on the 8 CE cosets x = 3 w_8n^r <w_n>
Fe8 ce_inv_zn(int log_n);
struct Openings;

}  // namespace zk

struct zk_prover {
    int device = 0;
    hipStream_t st = nullptr;
    // upload stream: a host-resident trace goes up here in column groups, each group's event gating its
    // interpolation and coset LDE on st (trace_lde_commit), so PCIe overlaps the group before it.  One stream per
    // device shared by all its provers (shared_upload_stream: the link is one resource, and the process then needs
    // P + 1 hardware queues for P provers instead of 2P; A/B at HIP's default 4 queues: 12.44 vs 12.64 ms per proof
    // for a stream per prover, profiles/r04_ab_queues_pass1.txt).
    // up_mu orders one prover's (copy, event) pairs against the other provers' on a shared stream.
    hipStream_t up = nullptr;
    std::mutex *up_mu = nullptr;
    // proofs in flight on this device (process-wide, beside the upload stream), and whether this proof started alone:
    // then trace_lde_commit takes the latency schedule (upload_sched: zk_prover_set_upload_schedule; AUTO: the
    // latency schedule iff no other proof is in flight on the device)
    std::atomic<int> *dev_busy = nullptr;
    bool lat_sched = false;
    int last_sched = 0;  // the schedule the last host-column proof ran (zk_prover_proof_info), 0 otherwise
    int upload_sched = ZK_SCHED_AUTO;  // zk_prover_set_upload_schedule
    // ... each group's event gating its kernels on st.  Measured (tools/ubench/upload_probe.hip): an event recorded
    // between the 16 MiB column copies of one stream halves their rate (29.7 vs 55 GB/s), but not between 112 MiB
    // copies (56.8 GB/s), so contiguous columns go up as one copy per group.  (Stream write / wait-value packets
    // avoid the slowdown too, but a compute stream parked on a wait-value packet can deadlock the copy stream's
    // write when the runtime maps both streams onto one hardware queue -- it hung under rocprofv3 --pmc.)
    hipEvent_t ev_up[zk::ZK_UPLOAD_GROUPS_MAX] = {};
    size_t max_n = 0;
    // 0: a full prover (every entry point).  G in {2, 4, 8}: sized for one rank of a G-way coset-sharded proof
    // (zk_prover_create_shard): the LDE-domain buffers hold the rank's 8/G cosets only, so it serves
    // zk_prove_sharded with that world size and nothing else.  (G = 1 is a full prover.)
    int shard_world = 0;
    uint32_t max_b = 0;
    zk::DeviceArena arena;
    fe *d_trace = nullptr, *polys = nullptr, *tmp = nullptr, *lde = nullptr, *comp = nullptr, *ctmp = nullptr,
       *cpolys = nullptr, *clde = nullptr, *deep = nullptr, *fri = nullptr;
    fe *ulde = nullptr;      // LDE of the DEEP polynomial (B*n, coset-major)
    fe *dscratch = nullptr;  // DEEP division scratch (power tables, suffix-sum inputs, coefficients)
    fe *x_ulde = nullptr, *x_dscratch = nullptr;  // the same for FieldExtension::Quadratic
    uint8_t *leaves = nullptr, *nodes = nullptr, *cleaves = nullptr, *cnodes = nullptr, *fri_dig = nullptr;
    fe *partials = nullptr, *ood_tab = nullptr, *ood = nullptr, *gather_out = nullptr;
    uint64_t *gather_idx = nullptr;
    // Pinned host staging for the small transfers on a proof's critical path (constants up; roots, the
    // degree flag, OOD values, FRI results down).  hipMemcpyAsync from or to pageable memory is staged
    // synchronously by the runtime (~20 us each between kernels); from pinned memory it is a DMA in
    // stream order (uploads); reads are copied by one kernel at d2h_flush time, so a read's device source
    // must stay unchanged from d2h_small until that flush.  Bump-allocated and rewound only by d2h_flush, after a stream sync, so no region is
    // reused while a copy from it may still be in flight.
    struct PendingRead {
        void *dst;              // caller's host destination (written by d2h_flush)
        uint8_t *stage;         // pinned staging slot the copy kernel writes
        const uint8_t *src;     // device source
        size_t len;
    };
    uint8_t *h_io = nullptr;
    size_t io_cap = 0, io_used = 0;
    std::vector<PendingRead> io_pending;
    uint64_t *h_gather_idx = nullptr;  // pinned host staging of the opening addresses / values
    fe *h_gather_out = nullptr;
    // pinned staging of the device trace generator's upload (vm_gpu.hip: chunk states, inputs, last row), grown
    // on demand
    uint8_t *h_vm = nullptr;
    size_t h_vm_cap = 0;
    hipEvent_t ev_vm = nullptr;  // recorded behind the last upload from h_vm (it is rewritten only once that is done)
    bool ev_vm_live = false;
    // zk_vm_prove: the preprocessed columns' polys / LDE and their BLAKE3 blocks 0 .. fix_prefix_blocks - 1 were
    // enqueued before the host stack pass (fixed_prefix); the next prove_fixed skips them.  Cleared by zk_vm_prove on
    // every way out.
    int fix_prefix_blocks = 0;
    zk::Openings *open = nullptr;      // per-proof openings, storage kept across proofs
    std::vector<uint8_t> proof_bytes;  // the serialized proof, storage kept across proofs
    unsigned *flag = nullptr;
    void *air_consts = nullptr, *deep_consts = nullptr, *fold_consts = nullptr;
    uint8_t *fri_seed = nullptr;  // device FRI coin state (32 B)
    fe *fri_alphas = nullptr;     // the alphas the device coin drew (2 per layer)
    fe_ws *fix_ws = nullptr;      // zk_vm_prove: the W sets of the last-row values of the preprocessed columns
    unsigned *sp_nz = nullptr;    // sparse-column flags of the current trace (SparseCols), W entries + 2W width flags
    fe *sp_last = nullptr;        // ... and the trace's last row
    // Hints (host-resident traces, prove_impl): the columns the previous proof of the same trace length AND program
    // (zk_pub_inputs::program_hash: column classes are a property of the program) found sparse are taken as sparse from
    // their last row alone and never uploaded; host threads check them during the proof (sp_bad: the hinted columns
    // that were not sparse; the proof is then redone without hints).  Narrow hint: the columns found to hold 8-bit
    // (nw8) or 32-bit (nw32) values in rows 0 .. n-2 are packed by host threads (which check every value: a column that
    // does not fit goes up whole instead) and go up as 1 or 4 bytes per element (h_pack, pinned), expanded on the
    // device.  One HintSet per (n, program), ZK_HINT_SETS of them, least recently used evicted: a server alternating
    // programs of one length keeps every program's hints instead of voiding each other's proofs (each refuted hint
    // costs a redone proof: hint_redos).
    struct HintSet {
        size_t n = 0;          // 0: an empty slot
        uint8_t key[32] = {};  // the program hash
        bool have = false;     // sparse / nw8 / nw32 hold a completed proof's findings
        uint32_t sparse = 0, nw8 = 0, nw32 = 0;
        bool clk_off = false;  // this (n, program)'s traces refuted the clock derivation: not speculated again
        uint64_t used = 0;     // LRU stamp
    };
    static constexpr int ZK_HINT_SETS = 8;
    HintSet hint_sets[ZK_HINT_SETS];
    uint64_t hint_stamp = 0;
    uint32_t hint_redos = 0;  // proofs voided by a refuted hint and redone (zk_prover_proof_info)
    uint32_t sp_hinted = 0, sp_bad = 0;
    bool sp_used = false;  // the last trace_lde_commit ran the detection (its flags are in sp_h)
    unsigned *sp_h = nullptr;  // pinned: the detection's flags, [0, W) nonzero, [W, 2W) 8-bit, [2W, 3W) 32-bit
    uint8_t *h_pack = nullptr;
    size_t h_pack_cap = 0;
    uint64_t up_bytes = 0;                        // zk_prover_upload_stats of the last host-column proof
    uint32_t up_sparse = 0, up_nw8 = 0, up_nw32 = 0;
    // Clock column (host-resident traces, trace_lde_commit): column 0 derived from the AIR's clock instead of
    // uploaded and transformed (clk_used: the last proof did; clk_bad: the host check refuted it; HintSet::clk_off: a
    // (length, program) whose traces refuted it, not speculated again)
    bool clk_used = false, clk_bad = false;
    // Virtual columns of the last host-trace commitment (trace_lde_commit): hinted sparse columns no constraint reads,
    // whose LDE is never written -- the row hashing and the openings form their values from the last row and e_(n-1)'s
    // LDE (virt_lagr) instead
    uint32_t virt = 0;
    fe virt_last[28] = {};
    const fe *virt_lagr = nullptr;
    // Sharded host-trace hints (shard.hip S2): the sparse columns and the clock a previous sharded proof of this length
    // and world found (from all-gathered flags, so every rank holds the same), checked by the ranks' host threads
    uint32_t sh_sparse = 0, sh_nw8 = 0, sh_nw32 = 0;  // (and the narrow ones: the owner rank uploads them packed)
    bool sh_clock = false;
    size_t sh_hint_n = 0, sh_clock_off_n = 0;
    int sh_hint_g = 0;
    uint8_t sh_hint_key[32] = {};  // ... for this program (zk_pub_inputs::program_hash)
    // coset-sharded proving (shard.hip), allocated on first use
    fe *sh_buf = nullptr;       // world x ZK_GATHER_CAP opened chunks (all-gathered)
    fe *sh_xr = nullptr;        // 3 * w_N^r of the local cosets
    fe *sh_zero = nullptr;      // one zero chunk (stands in for openings another rank owns)
    uint8_t *sh_roots = nullptr;  // world subtree roots
    // the block levels (0 .. log2 Bl) of the trace, composition and FRI layer-0 trees over this rank's cosets
    // (shard.hip DistTree): (2 Bl - 1) x n digests for the row trees, (2 Bl - 1) x n / 2 for layer 0 (fold >= 2)
    uint8_t *sh_blk = nullptr, *sh_cblk = nullptr, *sh_fblk = nullptr;
    uint8_t *sh_f1blk = nullptr;  // ... and FRI layer 1's, (2 Bl - 1) x n / 4 (committed on every rank, shard.hip S6)
    unsigned *sh_flags = nullptr;  // world degree flags
    // FieldExtension::Quadratic working set (planar E buffers), allocated on first use
    fe *x_comp = nullptr, *x_ctmp = nullptr, *x_clde = nullptr, *x_deep = nullptr, *x_fri = nullptr,
       *x_partials = nullptr, *x_tab = nullptr;
    void *x_air = nullptr, *x_deep_consts = nullptr, *x_fold_consts = nullptr;
    uint32_t *pow_seed = nullptr;            // grinding: the coin seed ...
    unsigned long long *pow_best = nullptr;  // ... and the smallest nonce found
    std::map<std::pair<int, int>, std::unique_ptr<zk::Plan>> plans;
    // stage timing
    // stage timing: events from a pool kept across proofs (creating ~11 events per proof cost host time
    // at the transcript round trips); the times are read only when asked for (zk_prover_stage_times)
    std::vector<hipEvent_t> stage_pool;
    std::vector<const char *> stage_names;  // stage_names[i] ends at event stage_pool[i]
    bool stage_done = false;                // the last proof completed: its events may be read
    std::vector<std::pair<const char *, float>> stage_ms;
    // exchanges of the last sharded proof (shard.hip xchg_start / xchg_wait): name, collective, bytes this rank
    // received from the other ranks, and the events bracketing the collective on the stream it ran on (ev, ev + 1)
    // and the compute stream's wait for it (ev + 2, ev + 3: the exposed time), pooled like the stage events
    struct XchgRec {
        const char *name;
        double bytes;
        size_t ev;
        int op;       // 0 all-to-all, 1 all-gather
        bool waited;  // the compute streams have waited for it (xchg_wait)
    };
    std::vector<hipEvent_t> xchg_pool;
    size_t xchg_next = 0;  // next free event of the pool (this proof)
    std::vector<XchgRec> xchg;
    // the sharded proof's schedule on local rank 0 (zk_prover_shard_schedule: the dependency order the library issued,
    // for tools/shard_model.py): entries in program order -- kind 'S' an exchange started, 'W' the compute stream
    // waits for one, 'K' a segment boundary -- each with the events recorded on the compute stream just before (pre)
    // and after (post) it; the compute segment before an entry spans [post of the previous entry, pre of this one],
    // and `lead` marks segments only the lead rank (local rank 0 of each process) runs
    struct SchedEnt {
        char kind;
        int x;  // exchange index (S, W)
        size_t pre, post;
        bool lead;  // the segment ENDING at this entry ran on the lead rank only
    };
    std::vector<SchedEnt> sched;
    int sched_world = 0;
    bool sched_measure = false;  // recorded in the serialised measurement mode (zk_comm_set_measure)
    hipStream_t cst = nullptr;     // sharded proofs: the exchanges' stream (created on first use)
    hipEvent_t ev_ready = nullptr;  // ... and the event that orders an exchange after this rank's compute stream
    // kernel stats (names / totals of the last profile)
    std::vector<std::string> kstat_names;
    std::vector<float> kstat_ms;
    std::vector<int> kstat_n;
    std::vector<double> kstat_bytes;
    std::vector<double> kstat_muls, kstat_addsubs;
    size_t last_n = 0;
    uint32_t last_b = 0;
};

namespace zk {

// One proof in flight on a device (zk_prover::dev_busy, process-wide per device) for the lifetime of the object;
// `others` = the proofs already in flight when it started.  The single-GPU AUTO upload schedule reads it (prove_once);
// sharded proofs count themselves on each local prover's device.
struct DeviceBusy {
    std::atomic<int> *b;
    int others;
    explicit DeviceBusy(std::atomic<int> *x) : b(x), others(x ? x->fetch_add(1) : 0) {}
    ~DeviceBusy() {
        if (b) b->fetch_sub(1);
    }
    DeviceBusy(const DeviceBusy &) = delete;
    DeviceBusy &operator=(const DeviceBusy &) = delete;
};

// Upload gating (trace_lde_commit, shard.hip S2): the host thread waits for upload event ev before it enqueues the
// kernels that read the group (the next group's copy is already queued).  The compute stream never parks on a
// cross-stream wait, which with fewer hardware queues than streams holds up the kernels of whatever stream shares its
// queue (A/B at 4 queues, 4 provers: 11.77 vs 11.99 ms per proof for a device-side stream wait;
// profiles/r04_ab_queues.txt).
int upload_gate(zk_prover *p, hipEvent_t ev);
// wait until every upload this prover has enqueued has completed (the caller's host buffers are free again)
void upload_drain(zk_prover *p);

// The event that closes one upload item on the shared upload stream (taken under up_mu).  record() records it and
// reports the status; an item left early by a failed copy records it from the destructor, so the copies already
// queued for the item are covered by an event upload_drain waits for.
struct UploadEvent {
    hipEvent_t ev;
    hipStream_t st;
    bool done = false;
    int record() {
        done = true;
        ZK_CHECK_HIP(hipEventRecord(ev, st));
        return ZK_OK;
    }
    ~UploadEvent() {
        if (!done) (void)hipEventRecord(ev, st);
    }
};

// vm::prove's preprocessed trace columns (vm_gpu.hip, zk_vm_prove).  Columns 0..11 (clk, opcode bits, hash flag,
// sponge, stack depth) depend on the program and lwe_size only, and a stack register column 12 + i with i >= the
// program's maximum depth is zero: every such column c is f_c + last[c] e_(n-1), with f_c fixed per program (f_c = 0
// for the zero registers) and last[c] the random last row.  Interpolation and coset LDE are linear, so its
// coefficients and LDE are f_c's (computed once per program) plus last[c] times those of e_(n-1) (the Lagrange
// basis polynomial of the last row): one streaming pass instead of 1 + B size-n NTTs per column.
struct FixedCols {
    int md;                  // trace columns 12 .. 12 + md - 1 are the dynamic ones (stack registers within depth)
    const fe *fpolys;        // 12 x n coefficients of f_0 .. f_11 (column-major)
    const fe *flde;          // 12 x B n, coset-major like the prover's LDE
    const fe *lagr;          // n coefficients of e_(n-1)'s interpolant
    const fe *lagr_lde;      // B n, coset-major
    fe last[W];              // the last row
};
// zk_prove_device of p->d_trace (whose dynamic columns hold the trace) with the preprocessed columns of fx
// Sparse trace columns (SparseCols) for this proof: allocates the flags on first use and clears them on p->st; *sp
// stays null when ZK_SPARSE=0 or the plan is too small for the four-step NTT.
int sparse_begin(zk_prover *p, Plan *pl, SparseCols *out, const SparseCols **sp);
int prove_fixed(zk_prover *p, size_t n, const zk_options *opt, const zk_pub_inputs *pub, const FixedCols *fx,
                uint8_t *proof_out, size_t *proof_len);
// polys / lde of the preprocessed columns (all but 12 .. 12 + md - 1): f_c + last[c] e_(n-1) (vm_gpu.hip); B: the LDE
// cosets held (fx's flde / lagr_lde and lde alike)
void fixed_axpy(hipStream_t st, const FixedCols &fx, const fe_ws *ws_dev, size_t n, size_t B, fe *polys, fe *lde);
// zk_vm_prove, before its host stack pass: fixed_axpy of fx into p->polys / p->lde and the BLAKE3 blocks of the rows'
// first columns that hold no live stack register (0 .. 2: columns 0 .. 11), on p->st; sets p->fix_prefix_blocks
int fixed_prefix(zk_prover *p, size_t n, uint32_t B, const FixedCols &fx);
// Host-trace column classes shared by the single-GPU and the sharded prover (prover.hip): ZK_SPARSE / ZK_CLOCK
// switches, the identity column's tables of a plan (the AIR clock: built once), and the host checks of a column's
// rows [r0, r1): all zero, or row i holding i
bool sparse_on();
bool clock_on();
bool narrow_on();
// rows [r0, r1) of a host column as `width`-byte integers (1 or 4) at dst + width * row; false if a value does not fit
bool pack_rows(const uint8_t *col, size_t r0, size_t r1, int width, uint8_t *dst);
int clock_tables(zk_prover *p, Plan *pl);
bool zero_rows(const uint8_t *col, size_t r0, size_t r1);
bool clock_rows(const uint8_t *col, size_t r0, size_t r1);
// zk_prove_sharded, and with `fixed` (one FixedCols per local rank, its own cosets; trace must be null) the sharded
// proof of zk_vm_prove_sharded's device traces (shard.hip)
int prove_sharded_entry(zk_comm *comm, zk_prover **provers, int nlocal, const uint8_t *trace, size_t n,
                        const zk_options *opt, const zk_pub_inputs *pub, uint8_t *proof_out, size_t *proof_len,
                        zk_record *rec, const FixedCols *fixed);
// the rank of local prover l of a sharded proof over comm
int shard_rank_of(const zk_comm *comm, int l);

// the single-GPU prove path (prover.hip) for a sharded proof over one rank: trace = host column-major trace, or
// NULL when it already sits in p->d_trace
int prove_single(zk_prover *p, const uint8_t *trace, size_t n, const zk_options *opt, const zk_pub_inputs *pub,
                 uint8_t *proof_out, size_t *proof_len, zk_record *rec);

// ---- small transfers through the pinned staging area (zk_prover::h_io)
inline uint8_t *io_take(zk_prover *p, size_t len) {
    const size_t a = (len + 63) & ~(size_t)63;
    if (p->io_used + a > p->io_cap) return nullptr;
    uint8_t *r = p->h_io + p->io_used;
    p->io_used += a;
    return r;
}
// enqueue host -> device from a pinned copy of src (src may be reused as soon as this returns)
inline int h2d_small(zk_prover *p, void *dst_dev, const void *src, size_t len) {
    uint8_t *s = io_take(p, len);
    if (!s) ZK_FAIL(ZK_ERR_OUT_OF_MEMORY, "pinned staging area exhausted");
    memcpy(s, src, len);
    ZK_CHECK_HIP(hipMemcpyAsync(dst_dev, s, len, hipMemcpyHostToDevice, p->st));
    return ZK_OK;
}
// queue a device -> host read of len bytes (len % 4 == 0, src 4-byte aligned); dst is written by the
// next d2h_flush.  Nothing is enqueued yet: the flush copies every pending read in one kernel, so src_dev must
// hold the value to read until that flush (no later kernel in the stream may overwrite it before then).
inline int d2h_small(zk_prover *p, void *dst, const void *src_dev, size_t len) {
    if ((len & 3) || ((uintptr_t)src_dev & 3)) ZK_FAIL(ZK_ERR_INVALID_ARG, "d2h_small: unaligned read");
    if (p->io_pending.size() >= ZK_COPY_LIST_MAX) ZK_FAIL(ZK_ERR_OUT_OF_MEMORY, "too many pending reads");
    uint8_t *s = io_take(p, len);
    if (!s) ZK_FAIL(ZK_ERR_OUT_OF_MEMORY, "pinned staging area exhausted");
    p->io_pending.push_back({dst, s, (const uint8_t *)src_dev, len});
    return ZK_OK;
}
// Every pending read in one kernel (copy_to_host writes the pinned staging directly; the runtime's
// hipMemcpyAsync issued one blit kernel of ~4.5 us per read), one stream sync, then the host copies.
// The staging area starts over.
inline int d2h_flush(zk_prover *p) {
    if (!p->io_pending.empty()) {
        CopyList L;
        L.n = (int)p->io_pending.size();
        size_t words = 0;
        for (int i = 0; i < L.n; i++) {
            const auto &r = p->io_pending[i];
            L.src[i] = (const uint32_t *)r.src;
            L.dst[i] = (uint32_t *)r.stage;
            L.words[i] = (uint32_t)(r.len / 4);
            words = std::max(words, r.len / 4);
        }
        const hipError_t le = copy_to_host(p->st, L, words);
        if (le != hipSuccess) {
            (void)hipStreamSynchronize(p->st);
            p->io_pending.clear();
            p->io_used = 0;
            ZK_CHECK_HIP(le);
        }
    }
    const hipError_t e = hipStreamSynchronize(p->st);
    if (e == hipSuccess)
        for (const auto &r : p->io_pending) memcpy(r.dst, r.stage, r.len);
    // on a failed sync the destinations are not written (they may be gone once the caller returns)
    p->io_pending.clear();
    p->io_used = 0;
    ZK_CHECK_HIP(e);
    return ZK_OK;
}
// sync the prover's stream and start its staging area over (a sharded proof's non-lead provers only
// stage uploads, so they are rewound at the start of each proof)
inline int io_rewind(zk_prover *p) { return d2h_flush(p); }
// Scope guard for an entry point that stages transfers: whatever way the scope is left, reads still
// pending (an error return between d2h_small and d2h_flush) are dropped, never delivered later into
// the caller's stack or per-proof buffers, and the staging area starts over once the stream is idle.
struct IoScope {
    zk_prover *p;
    explicit IoScope(zk_prover *q) : p(q) { drop(); }
    ~IoScope() { drop(); }
    void drop() {
        if (p->io_pending.empty() && p->io_used == 0) return;
        (void)hipStreamSynchronize(p->st);
        p->io_pending.clear();
        p->io_used = 0;
    }
};


int get_plan(zk_prover *p, size_t n, uint32_t B, Plan **out);
void stage_begin(zk_prover *p);
void stage_mark(zk_prover *p, const char *name);
void stage_collect(zk_prover *p);
void collect_kernel_stats(zk_prover *p);

// ---------------------------------------------------------------- proof bytes and Merkle openings
struct Bytes {
    std::vector<uint8_t> v;
    void put(const void *d, size_t n) {
        const uint8_t *b = (const uint8_t *)d;
        v.insert(v.end(), b, b + n);
    }
    void u8(uint8_t x) { v.push_back(x); }
    void u16(uint16_t x) { put(&x, 2); }
    void u32(uint32_t x) { put(&x, 4); }
    void u64(uint64_t x) { put(&x, 8); }
};

// MerkleTree::prove_batch plan: which leaf / node digests, in serialization order [P12]
struct BatchPlan {
    std::vector<uint64_t> norm;                                // normalized (even, sorted, unique) leaf indexes
    std::vector<std::vector<std::pair<int, uint64_t>>> paths;  // per path: (0 = leaf, 1 = node, index)
    std::vector<uint64_t> cur, next;                           // planning scratch (kept for reuse)
    size_t count() const {
        size_t k = 0;
        for (auto &p : paths) k += p.size();
        return k;
    }
};
BatchPlan plan_batch(size_t nl, const std::vector<uint64_t> &idx);
void plan_batch(size_t nl, const std::vector<uint64_t> &idx, BatchPlan &out);  // reuses out's storage

// ---------------------------------------------------------------- protocol steps (host side)
// argument checks shared by every prove entry point; returns ZK_OK or a status (g_err set)
int check_prove_args(size_t n, size_t max_n, uint32_t max_b, const zk_options *opt, const zk_pub_inputs *pub);
// num_constraint_composition_columns for the ProcessorAir degrees [P5]
// S0: public coin seeded with Context::to_elements || PublicInputs::to_elements [P1]
Coin seed_coin(size_t n, const zk_options *opt, const zk_pub_inputs *pub);
// S3: composition coefficients (20 transition, 22 boundary) and the evaluator's constants [P3, P4]
void draw_air_consts(Coin &coin, const zk_pub_inputs *pub, size_t n, AirConsts &K, zk_record &R);
// FieldExtension::Quadratic: the coefficients are E values (a + bX); the composition is linear in them, so
// the evaluator runs once with the a components (Ka) and once with the b components (Kb)
void draw_air_consts_ext(Coin &coin, const zk_pub_inputs *pub, size_t n, AirConsts &Ka, AirConsts &Kb, zk_record &R);
// S5: record the OOD frame h = T(z) || T(zg) || H(z) and reseed the coin with its two hashes [P7]
void ood_reseed(Coin &coin, const fe *h, int C, zk_record &R);
// S5: DEEP coefficients and the combined constants k1, k2 [P8]
DeepConsts draw_deep_consts(Coin &coin, const fe *h, int C, fe z, fe zg, zk_record &R);
// FieldExtension::Quadratic versions [P15] (prover.hip): E working set on first use, OOD frame from the
// two-plane ood_eval_ext output, DEEP and fold constants, remainder from a planar last layer
int ensure_ext(zk_prover *p);
void ood_reseed_ext(Coin &coin, const std::vector<fe> &hv, int C, zk_record &R, std::vector<fe2> &e,
                    std::vector<fe> &h);
DeepConstsE draw_deep_consts_ext(Coin &coin, const std::vector<fe2> &e, int C, fe2 z, fe2 zg, zk_record &R);
FoldConstsE fold_consts_ext(fe2 alpha, uint32_t fold);
int remainder_step_ext(const std::vector<fe> &rv, uint32_t B, Coin &coin, zk_record &R, unsigned &degree_flag,
                       std::vector<fe> &rem_flat);
// S6: number of FRI layers for an LDE domain of N points [P9]
int fri_num_layers(size_t N, const zk_options *opt);
FoldConsts fold_consts(fe alpha, uint32_t fold);
// S6: interpolate the last layer (natural order, over 3 * <w_L>), keep L/B coefficients, commit [P9]
int remainder_step(std::vector<fe> &last, uint32_t B, Coin &coin, zk_record &R, unsigned &degree_flag);
// S7: grinding nonce (on the GPU of `p` for grinding >= 8, else on the host) and the sorted unique
// query positions [P10, P11]
int grind_and_positions(zk_prover *p, Coin &coin, const zk_options *opt, size_t N, zk_record &R,
                        std::vector<uint64_t> &pos);
// positions folded down the FRI layers, first-occurrence order [P12]
std::vector<std::vector<uint64_t>> fri_fold_positions(const std::vector<uint64_t> &pos, size_t N, uint32_t fold,
                                                      int nl);

// Everything the proof bytes contain besides the record: opened values and, per Merkle opening
// (trace, constraint, FRI layers), the batch plan and its digests in serialization order.
struct Openings {
    std::vector<fe> trace_rows, comp_rows;       // nu x W, nu x C
    std::vector<std::vector<fe>> fri_rows;       // per layer: |fri_pos[l]| x fold
    std::vector<BatchPlan> plans;                // 2 + nl
    std::vector<std::vector<uint8_t>> digests;   // 2 + nl, 32 B each, plan order
    void reset(size_t nplans) {  // keeps every vector's capacity
        trace_rows.clear();
        comp_rows.clear();
        fri_rows.resize(nplans - 2);
        plans.resize(nplans);
        digests.resize(nplans);
    }
};
// S9: Proof::to_bytes [P13, P14].  E values are k = opt->field_extension base elements each:
// ood_flat = [T(z)]_W ++ [T(zg)]_W ++ [H(z)]_C flattened, comp_rows nu x C*k, fri_rows |pos| x fold*k;
// the remainder is R.remainder (k = 1) or rem_flat (rem_len x k).
std::vector<uint8_t> serialize_proof(size_t n, const zk_options *opt, int C, const zk_record &R, const fe *ood_flat,
                                     const Openings &O, const std::vector<fe> *rem_flat = nullptr);
void serialize_proof(size_t n, const zk_options *opt, int C, const zk_record &R, const fe *ood_flat, const Openings &O,
                     const std::vector<fe> *rem_flat, std::vector<uint8_t> &out);  // into out (storage reused)
// copy the proof out (proof_len in/out) and fold the degree flag into the status
int deliver_proof(const std::vector<uint8_t> &bytes, unsigned degree_flag, uint8_t *proof_out, size_t *proof_len);

}  // namespace zk
