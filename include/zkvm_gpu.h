/*
 * zkvm_gpu.h -- C ABI of the MI355X (gfx950) STARK prover for the Encrypt-zkVM execution trace.
 *
 * Drop-in boundary: every entry point below replaces one piece of the reference's
 * `impl winterfell::Prover for ExecutionProver` (prover/src/lib.rs:40-77) as driven by
 * `vm::prove` (vm/src/lib.rs:13-29).  The reference Rust host would bind these through a
 * thin FFI (see INTEGRATION.md for the cgo-style/Rust `extern "C"` stubs).
 *
 * Conventions
 *  - Field elements are winterfell f128 values (p = 2^128 - 45*2^40 + 1), canonical,
 *    16 bytes little-endian each (the `f128::BaseElement` byte format).
 *  - Trace matrices are column-major: column c occupies bytes [c*n*16, (c+1)*n*16).  The
 *    column order is the one `Processor::trace` emits (vm/src/processor/mod.rs:76-84):
 *    clk, 5 opcode bits, hash flag, 4 sponge words, stack depth, 16 stack registers (28 total).
 *  - All functions return ZK_OK (0) or a negative status, never abort, and leave a message
 *    for zk_last_error() (thread-local).  Buffers are owned by the caller.
 *  - A zk_prover owns one GPU's device memory and one HIP stream.  Calls on one prover are not
 *    reentrant; different provers may be used from different threads concurrently.
 */
#ifndef ZKVM_GPU_H
#define ZKVM_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZK_OK 0
#define ZK_ERR_INVALID_ARG -1
#define ZK_ERR_BUFFER_TOO_SMALL -2
#define ZK_ERR_DEVICE -3
#define ZK_ERR_OUT_OF_MEMORY -4
#define ZK_ERR_PROGRAM -10  /* ProgramError (vm/src/program/errors.rs) */
#define ZK_ERR_STACK -11    /* StackError (vm/src/processor/errors.rs:4-42) */
#define ZK_ERR_CHIPLETS -12 /* ChipletsError (vm/src/processor/errors.rs:44-71) */
#define ZK_ERR_DEGREE -20   /* proof written, but the trace does not satisfy ProcessorAir */
#define ZK_ERR_VERIFY -30   /* zk_verify: the proof is rejected (reason in msg) */

#define ZK_TRACE_WIDTH 28
#define ZK_MAX_COLS 32
#define ZK_MAX_TCONS 32
#define ZK_MAX_ASSERTS 32
#define ZK_MAX_CCOLS 16
#define ZK_MAX_FRI_LAYERS 16
#define ZK_MAX_REMAINDER 256
#define ZK_MAX_QUERIES 255

/* ProofOptions::new(num_queries, blowup, grinding, field_extension, fri_folding, fri_rem_max_deg)
 * -- the reference hard-codes (32, 8, 0, None, 8, 127) at vm/src/lib.rs:20.
 * field_extension: 1 = FieldExtension::None, 2 = FieldExtension::Quadratic; 3 (Cubic) is refused
 * with ZK_ERR_INVALID_ARG (winter-math implements no cubic extension of f128). */
typedef struct {
    uint32_t num_queries;
    uint32_t blowup;
    uint32_t grinding;
    uint32_t field_extension;
    uint32_t fri_folding;
    uint32_t fri_rem_max_deg;
} zk_options;

/* air::PublicInputs (air/src/lib.rs:18-47) plus the two ServerKey values the constraints use
 * (lwe_size = k + 1, delta = q / p; fhe/src/server_key.rs:78-124, fhe/src/parameters.rs:17).
 * The reference also carries the ServerKey's secret bits here; the constraints never read them. */
typedef struct {
    uint8_t program_hash[2][16];
    uint8_t stack_outputs[16][16];
    uint32_t lwe_size;
    uint32_t delta;
} zk_pub_inputs;

/* Every deterministic intermediate of one proof (for stage-wise parity checks).  Same layout as
 * the oracle's or_record. */
typedef struct {
    uint32_t trace_len, lde_len, width, num_ccols, num_fri_layers, remainder_len;
    uint32_t num_positions;
    uint32_t _pad;
    uint8_t trace_root[32];
    uint8_t coeff_t[ZK_MAX_TCONS][16];
    uint8_t coeff_b[ZK_MAX_ASSERTS][16];
    uint8_t constraint_root[32];
    uint8_t z[16];
    uint8_t ood_trace_z[ZK_MAX_COLS][16];
    uint8_t ood_trace_zg[ZK_MAX_COLS][16];
    uint8_t ood_constraints[ZK_MAX_CCOLS][16];
    uint8_t deep_t[ZK_MAX_COLS][16];
    uint8_t deep_c[ZK_MAX_CCOLS][16];
    uint8_t fri_roots[ZK_MAX_FRI_LAYERS][32];
    uint8_t fri_alphas[ZK_MAX_FRI_LAYERS][16];
    uint8_t remainder[ZK_MAX_REMAINDER][16];
    uint8_t remainder_commitment[32];
    uint64_t pow_nonce;
    uint64_t positions[ZK_MAX_QUERIES + 1];
} zk_record;

/* Optional host copies of full-size intermediates (NULL = skip), natural LDE order. */
typedef struct {
    uint8_t *trace_polys;  /* 28 * n coefficients, column-major */
    uint8_t *trace_lde;    /* N * 28, row-major */
    uint8_t *trace_leaves; /* N * 32 */
    uint8_t *composition;  /* 8n evaluations over the constraint-evaluation domain */
    uint8_t *comp_polys;   /* c * n coefficients, column-major */
    uint8_t *comp_lde;     /* N * c, row-major */
    uint8_t *deep;         /* N evaluations */
    uint8_t *fri_layer1;   /* N / fold evaluations */
} zk_dump;

typedef struct zk_prover zk_prover;
typedef struct zk_trace_lde zk_trace_lde;

const char *zk_last_error(void);
int zk_device_count(int *count);

/* ---- the runtime this library is linked against (no reference counterpart: host plumbing) ----
 * The library needs libamdhip64.so.7 and librccl.so.1 (RUNPATH /opt/rocm/lib).  A host that also loads another
 * copy of either (PyTorch bundles its own) must load it first, or the process maps two HIP runtimes; these calls let a
 * host get what it needs from the copy the library uses instead.  zk_runtime_versions: hipRuntimeGetVersion and
 * ncclGetVersion of the mapped copies.  zk_device_pci_bus_id: "dddd:bb:dd.f" of a device (the host's NUMA binding
 * reads /sys/bus/pci/devices/<id>/numa_node).  zk_device_synchronize: hipDeviceSynchronize on one device (the bench's
 * barriers). */
int zk_runtime_versions(int *hip_runtime, int *rccl);
int zk_device_pci_bus_id(int device, char *bus_id, int len);
int zk_device_synchronize(int device);

/* ---- prover object: device memory sized for traces up to max_trace_len rows ----
 * Process-wide side effect: the first zk_prover_create on a device that the process has not used yet
 * sets hipDeviceScheduleSpin for that device, so every host thread waiting on a stream of that device
 * (this library's transcript round trips, and any other code's syncs) busy-spins instead of yielding
 * (-0.05 ms per 2^20 proof).  Set ZK_SPIN_WAIT=0 in the environment to keep the runtime's default. */
int zk_prover_create(int device, size_t max_trace_len, uint32_t max_blowup, zk_prover **out);
/* A prover sized for ONE rank of a `world`-way coset-sharded proof (zk_prove_sharded, blowup 8): the buffers of
 * the LDE domain (trace and composition LDE, DEEP, NTT scratch, Merkle subtrees) hold the rank's 8/world cosets
 * only -- about 12.6 GB per rank at 2^22, world 8, against 50 GB for a full prover.  It serves zk_prove_sharded
 * with that world size; every single-GPU entry point refuses it (ZK_ERR_INVALID_ARG). */
int zk_prover_create_shard(int device, size_t max_trace_len, int world, zk_prover **out);
void zk_prover_destroy(zk_prover *p);
/* Process-wide pool for callers that build a prover per proof, as the reference does (ExecutionProver::new inside
 * vm::prove, vm/src/lib.rs:24): zk_prover_acquire returns an idle pooled full prover of this device with at least
 * these sizes (the smallest such; its per-size tables are already built), else creates one; zk_prover_release hands
 * it back instead of freeing its ~12.5 GB (2^20).  Thread-safe.  zk_prover_pool_trim frees the idle provers of one
 * device (-1: every device) and returns how many. */
int zk_prover_acquire(int device, size_t max_trace_len, uint32_t max_blowup, zk_prover **out);
void zk_prover_release(zk_prover *p);
int zk_prover_pool_trim(int device);
/* device pointer to a scratch region large enough for a 28 x max_trace_len trace (so callers can
 * stage a device-resident trace without their own allocator) */
int zk_prover_trace_buffer(zk_prover *p, void **d_trace);

/* Prover::prove (vm/src/lib.rs:26 -> winterfell generate_proof), whole proof.
 * Host trace variant: trace is 28 x n, column-major, host memory.  The trace goes up in column groups on
 * a copy stream, each group's interpolation and coset LDE starting as soon as it is in HBM.  From
 * page-locked memory (zk_host_alloc / zk_host_register) the copies are DMAs at the link rate; pageable
 * memory works too, staged by the HIP runtime at a lower rate.  The trace is not read after return. */
int zk_prove(zk_prover *p, const uint8_t *trace, size_t n, const zk_options *opt, const zk_pub_inputs *pub,
             uint8_t *proof_out, size_t *proof_len);
/* The same with one pointer per column (n * 16 bytes each): winterfell's ColMatrix / TraceTable keeps
 * every column in its own Vec<f128> (vm/src/lib.rs:18), which binds here without a flattening copy. */
int zk_prove_columns(zk_prover *p, const uint8_t *const *columns, size_t n, const zk_options *opt,
                     const zk_pub_inputs *pub, uint8_t *proof_out, size_t *proof_len);
/* ... with the optional record / dumps of zk_prove_device */
int zk_prove_columns_ex(zk_prover *p, const uint8_t *const *columns, size_t n, const zk_options *opt,
                        const zk_pub_inputs *pub, uint8_t *proof_out, size_t *proof_len, zk_record *rec,
                        const zk_dump *dump);
/* Page-locked host memory for traces (hipHostMalloc, usable from every device), e.g. the buffer the
 * VM writes its trace into (zk_vm_trace), and page-locking of a caller's own buffer (hipHostRegister:
 * costs about as much as one copy of it, so register buffers that are reused). */
int zk_host_alloc(size_t bytes, void **ptr);
void zk_host_free(void *ptr);
int zk_host_register(void *ptr, size_t bytes);
int zk_host_unregister(void *ptr);
/* Device trace variant (trace already resident in HBM on this prover's device), with optional
 * record / dumps.  proof_len is in/out: capacity in, bytes written out; ZK_ERR_BUFFER_TOO_SMALL
 * reports the needed size. */
int zk_prove_device(zk_prover *p, const void *d_trace, size_t n, const zk_options *opt, const zk_pub_inputs *pub,
                    uint8_t *proof_out, size_t *proof_len, zk_record *rec, const zk_dump *dump);

/* ---- plug point 1: Prover::new_trace_lde (prover/src/lib.rs:55-62) -> DefaultTraceLde ---- */
/* interpolate the trace, extend it over the blowup coset domain and commit to its rows.
 * The LDE lives in the prover's device memory until zk_lde_free. */
int zk_lde_new(zk_prover *p, const uint8_t *trace, size_t width, size_t n, uint32_t blowup, zk_trace_lde **out,
               uint8_t root[32]);
/* TraceLde::read_main_trace_frame_into: rows lde_step and (lde_step + blowup) mod N */
int zk_lde_read_frame(zk_trace_lde *lde, size_t lde_step, uint8_t *cur, uint8_t *next);
/* TraceLde::query: rows at positions (width elements each) + batch Merkle proof bytes */
int zk_lde_query(zk_trace_lde *lde, const uint64_t *positions, size_t k, uint8_t *rows_out, uint8_t *proof_out,
                 size_t *proof_len);
void zk_lde_free(zk_trace_lde *lde);

/* ---- plug point 2: Prover::new_evaluator (prover/src/lib.rs:65-72) + evaluate ----
 * DefaultConstraintEvaluator over ProcessorAir: coeff_t = 20 transition coefficients,
 * coeff_b = 22 boundary coefficients (assertions sorted by (stride, step, column));
 * out receives the 8n composition-trace values in natural CE-domain order. */
int zk_eval_constraints(zk_trace_lde *lde, const zk_pub_inputs *pub, const uint8_t *coeff_t, const uint8_t *coeff_b,
                        uint8_t *out);

/* ---- plug point 3: Prover::build_constraint_commitment (winterfell 0.9 provided method;
 * SURVEY.md 8(b); its input is the CompositionPolyTrace new_evaluator's evaluate returns,
 * prover/src/lib.rs:65-72) ----
 * composition: the 8n values zk_eval_constraints writes (natural CE-domain order).  Interpolates them
 * over the CE coset, splits the polynomial into num_cols column polynomials of n coefficients
 * (CompositionPoly; polys_out, optional: num_cols x n, column-major), extends each over the trace
 * LDE's blowup coset domain and commits to the rows (ConstraintCommitment; root).  Returns
 * ZK_ERR_DEGREE (no handle) when the polynomial has a coefficient at or beyond num_cols * n.  The
 * handle reads the prover's device memory: valid until the next proof or commitment on that prover. */
typedef struct zk_comp_commit zk_comp_commit;
int zk_commit_composition(zk_trace_lde *lde, const uint8_t *composition, uint32_t num_cols, zk_comp_commit **out,
                          uint8_t root[32], uint8_t *polys_out);
/* ConstraintCommitment::query: rows (num_cols elements each) at positions + batch Merkle proof bytes */
int zk_comp_query(zk_comp_commit *comp, const uint64_t *positions, size_t k, uint8_t *rows_out, uint8_t *proof_out,
                  size_t *proof_len);
void zk_comp_free(zk_comp_commit *comp);

/* ---- one proof sharded over several GPUs ----
 * The LDE domain is split by coset: rank g of `world` (1, 2, 4 or 8; blowup 8) owns the block of cosets
 * g * 8/world .. (g + 1) * 8/world - 1.  Exchanges (Merkle block nodes, composition coefficient slices, FRI layer 1,
 * openings)
 * go through a zk_comm: RCCL over xGMI with one process per GPU (zk_comm_unique_id on rank 0,
 * shared out of band, then zk_comm_create_rccl on every rank), or an in-process loopback that drives
 * every rank from one process (tests; one prover per rank), or a caller transport (zk_comm_create_host).
 * Every rank passes the same host trace (column-major, 28 x n x 16 B; rank g reads and uploads only
 * columns g, g + world, g + 2 world, ... and receives the other columns' polynomials from their owners),
 * or NULL: the whole trace already sits in each prover's zk_prover_trace_buffer.  Every rank receives
 * the same proof bytes, identical to zk_prove's. */
typedef struct zk_comm zk_comm;
int zk_comm_create_loopback(int world, zk_comm **out);
int zk_comm_unique_id(uint8_t id[128]);
int zk_comm_create_rccl(const uint8_t id[128], int rank, int world, int device, zk_comm **out);
/* A communicator over a caller-supplied transport (MPI, gloo, TCP; also across nodes): one rank per process.
 * For every exchange the library copies this rank's device chunk(s) to host memory, calls fn, and copies recv
 * back to the device.  op ZK_XCHG_ALL_TO_ALL: send holds `world` chunks of `bytes` (chunk d is for rank d), recv
 * receives `world` chunks (chunk s came from rank s); op ZK_XCHG_ALL_GATHER: send is one chunk of `bytes`, recv
 * receives the `world` chunks in rank order.  fn returns 0 on success (anything else fails the proof with
 * ZK_ERR_DEVICE); every rank calls it the same number of times with the same op and bytes. */
typedef int (*zk_exchange_fn)(void *ctx, int op, const void *send, void *recv, size_t bytes);
enum { ZK_XCHG_ALL_TO_ALL = 0, ZK_XCHG_ALL_GATHER = 1 };
int zk_comm_create_host(int rank, int world, zk_exchange_fn fn, void *ctx, zk_comm **out);
void zk_comm_destroy(zk_comm *comm);
/* Measurement mode of a loopback communicator (tools/shard_model.py): every rank's kernels and the exchange copies
 * run on ONE stream in program order, so each compute segment of the schedule (zk_prover_shard_schedule) is the
 * ranks' compute alone, serialised (no overlap, no exchange time inside); the proof bytes are unchanged.  on = 0
 * returns to the normal mode (exchanges on their own stream, overlapped with compute).  Refused for RCCL and
 * host-exchange communicators. */
int zk_comm_set_measure(zk_comm *comm, int on);
/* The trace interpolation's split when the trace is already in every rank's HBM (trace = NULL, zk_vm_prove_sharded):
 * `replicated` of the columns to interpolate are interpolated and extended by every rank itself, at the start, under
 * the first two coefficient all-gathers; the others are split round robin and all-gathered.  -1 (the default): the
 * library's choice (four columns), from tools/shard_model.py's replay of measured schedules.
 * Same proof bytes for every value. */
int zk_comm_set_trace_split(zk_comm *comm, int replicated);
int zk_prove_sharded(zk_comm *comm, zk_prover **provers, int nlocal, const uint8_t *trace, size_t n,
                     const zk_options *opt, const zk_pub_inputs *pub, uint8_t *proof_out, size_t *proof_len,
                     zk_record *rec);
/* The collectives of the last sharded proof on this (local rank 0) prover, aggregated by name (trace_coeffs,
 * trace_digests, trace_roots, comp_slices, comp_columns, degree_flags, comp_digests, comp_roots, ood_parts,
 * deep_totals, deep_slices, fri0_digests, fri0_roots, fri_layer1, openings): ms between HIP events recorded on the
 * stream the collective runs on around each call (waiting for slower ranks included), bytes this rank received from
 * the other ranks, and the number of calls.  Valid once the proof has returned, until the next proof. */
int zk_prover_exchange_stats(zk_prover *p, const char **names, float *ms, double *bytes, int *calls, int cap,
                             int *count);
/* The same with each collective's exposed time beside its total: exposed_ms is how long the compute stream waited
 * for it (events around the stream wait; 0 when the collective finished under the compute issued meanwhile).  The
 * collectives run on a stream of their own (round 6), so only what a stage waits for shows up as exposed. */
int zk_prover_exchange_stats_ex(zk_prover *p, const char **names, float *ms, float *exposed_ms, double *bytes,
                                int *calls, int cap, int *count);
/* The last sharded proof's schedule on this (local rank 0) prover, as JSON: the order in which the library started
 * exchanges, waited for them and ran the compute segments between (each segment's measured ms, and whether only the
 * lead rank ran it), for tools/shard_model.py.  *len = bytes needed (with the NUL); ZK_ERR_BUFFER_TOO_SMALL when
 * cap is short.  In the measurement mode (zk_comm_set_measure) the segments are the serialised ranks' compute. */
int zk_prover_shard_schedule(zk_prover *p, char *buf, size_t cap, size_t *len);
/* The host-to-device trace traffic of the last proof from host columns (zk_prove / zk_prove_columns): bytes copied,
 * the columns taken as sparse (zero but the last row: their last value only), and the columns uploaded packed as 8-
 * or 32-bit integers (narrow; each value checked on the host first).  Bit c = trace column c. */
int zk_prover_upload_stats(zk_prover *p, uint64_t *bytes, uint32_t *sparse_cols, uint32_t *narrow8_cols,
                           uint32_t *narrow32_cols);
/* the columns of the last host-column proof that were derived from the AIR instead of uploaded and transformed: bit 0,
 * the clock (rows 0 .. n-2 of any accepted trace hold 0 .. n-2: air/src/constrains.rs clock constraint and the
 * clk[0] = 0 assertion), checked against the caller's column by host threads */
int zk_prover_upload_derived(zk_prover *p, uint32_t *derived_cols);
/* How a host-resident trace goes up (zk_prove / zk_prove_columns).  ZK_SCHED_AUTO (the default): the latency schedule
 * for a proof that starts with no other proof in flight on its device, else the throughput schedule.
 * ZK_SCHED_THROUGHPUT: the narrow (packed) columns in two parts through the copy engine between 64-MB column groups.
 * ZK_SCHED_LATENCY: the first two column groups start crossing at once and the packed narrow columns are expanded by a
 * kernel reading the pinned bytes, in small parts, so the first kernels start ~0.2 ms into the call.  Same proof bytes.
 * (No reference counterpart: winterfell's prover has no upload; a tuning knob for servers.) */
enum { ZK_SCHED_AUTO = 0, ZK_SCHED_THROUGHPUT = 1, ZK_SCHED_LATENCY = 2 };
int zk_prover_set_upload_schedule(zk_prover *p, int schedule);
/* What the last proof on this prover did.  schedule: the upload schedule the last host-column proof ran
 * (ZK_SCHED_THROUGHPUT or ZK_SCHED_LATENCY; 0 after a device-trace proof).  The AUTO rule, as a contract: a proof takes
 * the latency schedule iff no other proof -- single-GPU or a rank of a sharded proof -- is in flight on its device
 * when it starts (a proof counts as in flight from entry until its uploads and kernels have drained).
 * hint_redos: proofs this prover voided and redid because a column hint was refuted (cumulative).  hint_sets: the
 * (trace length, program hash) column-hint sets it holds (at most 8, least recently used evicted).  hinted_sparse /
 * derived: the sparse columns (bit c) and derived columns (bit 0, the clock) the last proof took from its hints. */
typedef struct {
    int32_t schedule;
    uint32_t hint_redos;
    uint32_t hint_sets;
    uint32_t hinted_sparse;
    uint32_t derived;
    uint32_t _pad;
} zk_proof_info;
int zk_prover_proof_info(const zk_prover *p, zk_proof_info *out);

/* ---- verifier: winterfell::verify::<ProcessorAir, Blake3_256, DefaultRandomCoin> (vm/src/lib.rs:93-98)
 * for the proof layout above, on the host (no GPU needed).  min_security: conjectured bits required
 * (the reference's test asks 95 for its options).  Returns ZK_OK, or ZK_ERR_VERIFY with the reason in
 * msg. */
int zk_verify(const uint8_t *proof, size_t proof_len, const zk_pub_inputs *pub, uint32_t min_security, char *msg,
              size_t msg_cap);

/* ---- per-stage timing of the last proof (ms), for benchmarks ---- */
int zk_prover_stage_times(zk_prover *p, const char **names, float *ms, int cap, int *count);
/* per-kernel device time (HIP events on the prover's stream) and algorithmic HBM bytes accumulated
 * since the last reset; enabled by zk_prover_profile(p, 1).  Passing all-NULL arrays resets. */
int zk_prover_profile(zk_prover *p, int enable);
int zk_prover_kernel_stats(zk_prover *p, const char **names, float *total_ms, int *launches, double *total_bytes,
                           int cap, int *count);
/* the same kernels (same order) with their algorithmic f128 multiplies and additions/subtractions
 * (0 where a kernel's operation count is not modelled; the NTT passes are) */
int zk_prover_kernel_ops(zk_prover *p, double *total_muls, double *total_addsubs, int cap, int *count);

/* ---- VM trace generator (harness; vm::Processor::run + trace, vm/src/processor/mod.rs:61-95) ----
 * source: assembly text (Program::compile); public: u8 inputs; secret: ciphertexts of lwe_size
 * elements; last_row: the 28 values the reference draws from thread_rng().  trace_out receives
 * 28 x n column-major with n <= cap_rows; outputs = 16 stack values; hash = program hash.
 * trace_out = NULL is a size query: *n_out is set from the compiled program alone (the VM does not
 * run) and ZK_ERR_BUFFER_TOO_SMALL is returned. */
int zk_vm_trace(const char *source, const uint8_t *public_in, size_t num_public, const uint8_t *secret,
                size_t num_secret, uint32_t lwe_size, uint32_t delta, const uint8_t *last_row, uint8_t *trace_out,
                size_t cap_rows, size_t *n_out, uint8_t *outputs, uint8_t *program_hash);
/* The same in the reference's two steps.  zk_program_compile = Program::compile (vm/src/program/mod.rs:37-131):
 * parse, pad, hash; the handle keeps the chiplet's per-step sponge states the hash computation produced (they
 * depend on the code alone).  zk_program_trace = Processor::run + trace (vm/src/processor/mod.rs:61-95) of that
 * program on these inputs: the stack machine runs once sequentially (errors, chunk states), then threads
 * (ZK_VM_THREADS, else OMP_NUM_THREADS, else all cores) write the rows.  trace_out = NULL runs the program and
 * reports n (ZK_ERR_BUFFER_TOO_SMALL).  A compiled program may be traced from several threads at once. */
typedef struct zk_program zk_program;
int zk_program_compile(const char *source, zk_program **out, uint8_t *program_hash, size_t *trace_len);
int zk_program_trace(const zk_program *prog, const uint8_t *public_in, size_t num_public, const uint8_t *secret,
                     size_t num_secret, uint32_t lwe_size, uint32_t delta, const uint8_t *last_row,
                     uint8_t *trace_out, size_t cap_rows, size_t *n_out, uint8_t *outputs);
void zk_program_free(zk_program *prog);
const char *zk_vm_last_error(void);

/* ---- vm::prove (vm/src/lib.rs:13-29) with the trace written on the GPU ----
 * zk_vm_trace_device = Processor::run + output + trace (vm/src/processor/mod.rs:61-101) into the prover's own trace
 * buffer (zk_prover_trace_buffer, 28 x n column-major): the host runs the stack machine once (every error the
 * reference raises, with its status and text in zk_vm_last_error / zk_last_error; the 16 outputs) and uploads its
 * state every 64 rows plus the inputs (~6 MB at 2^20 instead of the 448 MiB trace); kernels replay the machine and
 * write the rows.  lwe_size must be in [1, 5] (the AIR's range).  last_row: the 28 values Processor::trace draws from
 * thread_rng() (mod.rs:86-92), or NULL to draw them here (uniform nonzero field elements).  Returns once the trace is
 * in HBM.  Works on every prover, a rank of a sharded proof included (then zk_prove_sharded with trace = NULL). */
int zk_vm_trace_device(zk_prover *p, zk_program *prog, const uint8_t *public_in, size_t num_public,
                       const uint8_t *secret, size_t num_secret, uint32_t lwe_size, uint32_t delta,
                       const uint8_t *last_row, size_t *n_out, uint8_t *outputs);
/* The whole of vm::prove on one GPU: the device trace above, then ExecutionProver::new(options, program hash,
 * outputs, server key) + prove (vm/src/lib.rs:20-26) on it -- the same proof bytes as zk_prove of the host VM's trace.
 * outputs (16 x 16 B) and program_hash (2 x 16 B) are optional outputs (the reference returns (hash, output, proof)). */
int zk_vm_prove(zk_prover *p, zk_program *prog, const uint8_t *public_in, size_t num_public, const uint8_t *secret,
                size_t num_secret, uint32_t lwe_size, uint32_t delta, const uint8_t *last_row, const zk_options *opt,
                uint8_t *proof_out, size_t *proof_len, uint8_t *outputs, uint8_t *program_hash);
/* vm::prove as ONE proof sharded over the ranks of `comm`: every local rank writes the trace into its
 * own HBM (zk_vm_trace_device: the host stack pass is repeated per process, no trace crosses PCIe or xGMI), then
 * zk_prove_sharded over the device traces.  last_row is REQUIRED (every rank must write the same trace; the caller
 * draws it once and broadcasts it).  The same proof bytes as zk_vm_prove / zk_prove of that trace, on every rank. */
int zk_vm_prove_sharded(zk_comm *comm, zk_prover **provers, int nlocal, zk_program *prog, const uint8_t *public_in,
                        size_t num_public, const uint8_t *secret, size_t num_secret, uint32_t lwe_size, uint32_t delta,
                        const uint8_t *last_row, const zk_options *opt, uint8_t *proof_out, size_t *proof_len,
                        uint8_t *outputs, uint8_t *program_hash);

#ifdef __cplusplus
}
#endif
#endif
