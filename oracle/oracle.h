/*
 * oracle.h -- CPU restatement ("oracle") of the Encrypt-zkVM STARK prove path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (encrypt-zkvm_amd/, include/) links,
 * loads or calls this code; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker.
 *
 * Parity status (see DESIGN.md "Oracle and parity"):
 *   - reference-crate code (vm/, air/, crypto/, fhe/ arithmetic): pinned by the reference's
 *     own tests, ported as known-answer tests in tests/test_oracle_*.py;
 *   - BLAKE3: pinned by published BLAKE3 test vectors;
 *   - winterfell 0.9.0 protocol layer (transcript, composition, DEEP, FRI, proof bytes):
 *     PARITY UNPINNED -- winterfell is not vendored in /root/reference and no Rust toolchain
 *     exists here; the restatement follows the published winterfell 0.9 design and every
 *     protocol choice is listed in DESIGN.md "Protocol profile".
 *
 * All field values cross this interface as 16-byte little-endian canonical integers
 * (the winterfell f128 wire format, crypto/src/rescue.rs:66-72 `Hash::to_bytes`).
 */
#ifndef ZKVM_ORACLE_H
#define ZKVM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_MAX_COLS 32
#define OR_MAX_TCONS 32
#define OR_MAX_ASSERTS 32
#define OR_MAX_CCOLS 16
#define OR_MAX_FRI_LAYERS 16
#define OR_MAX_REMAINDER 256
#define OR_MAX_QUERIES 255

/* status codes (shared numbering with include/zkvm_gpu.h) */
#define OR_OK 0
#define OR_ERR_INVALID_ARG -1
#define OR_ERR_BUFFER_TOO_SMALL -2
#define OR_ERR_PROGRAM -10
#define OR_ERR_STACK -11
#define OR_ERR_CHIPLETS -12
#define OR_ERR_DEGREE -20 /* proof written, but the trace does not satisfy the AIR */
#define OR_ERR_VERIFY -30

typedef struct {
    uint32_t num_queries;      /* ProofOptions::new arg 1 (vm/src/lib.rs:20) */
    uint32_t blowup;           /* arg 2 */
    uint32_t grinding;         /* arg 3 */
    uint32_t field_extension;  /* arg 4: 1 = None (only value supported) */
    uint32_t fri_folding;      /* arg 5 */
    uint32_t fri_rem_max_deg;  /* arg 6 */
} or_options;

typedef struct {
    uint8_t program_hash[2][16];  /* air/src/lib.rs:18-22 PublicInputs */
    uint8_t stack_outputs[16][16];
    uint32_t lwe_size;            /* ServerKey::lwe_size() = k + 1 */
    uint32_t delta;               /* LweParameters.delta = q / p */
} or_pub_inputs;

/* Every deterministic intermediate of one proof, for stage-wise parity checks. */
typedef struct {
    uint32_t trace_len, lde_len, width, num_ccols, num_fri_layers, remainder_len;
    uint32_t num_positions;
    uint32_t _pad;
    uint8_t trace_root[32];
    uint8_t coeff_t[OR_MAX_TCONS][16];
    uint8_t coeff_b[OR_MAX_ASSERTS][16];
    uint8_t constraint_root[32];
    uint8_t z[16];
    uint8_t ood_trace_z[OR_MAX_COLS][16];
    uint8_t ood_trace_zg[OR_MAX_COLS][16];
    uint8_t ood_constraints[OR_MAX_CCOLS][16];
    uint8_t deep_t[OR_MAX_COLS][16];
    uint8_t deep_c[OR_MAX_CCOLS][16];
    uint8_t fri_roots[OR_MAX_FRI_LAYERS][32];
    uint8_t fri_alphas[OR_MAX_FRI_LAYERS][16];
    uint8_t remainder[OR_MAX_REMAINDER][16];
    uint8_t remainder_commitment[32];
    uint64_t pow_nonce;
    uint64_t positions[OR_MAX_QUERIES + 1];
} or_record;

/* Optional full-size intermediates (NULL = not wanted). Sizes with N = blowup * n. */
typedef struct {
    uint8_t *trace_polys;   /* w * n coefficients, column-major */
    uint8_t *trace_lde;     /* N * w, row-major (natural LDE order) */
    uint8_t *trace_leaves;  /* N * 32 */
    uint8_t *composition;   /* N evaluations (CE domain = LDE domain) */
    uint8_t *comp_polys;    /* c * n coefficients, column-major */
    uint8_t *comp_lde;      /* N * c, row-major */
    uint8_t *deep;          /* N evaluations */
    uint8_t *fri_layer1;    /* N / fold evaluations (first folded layer), if any layer */
} or_dump;

/* ---- field (16-byte LE canonical) ---- */
void or_fadd(const void *a, const void *b, void *out);
void or_fsub(const void *a, const void *b, void *out);
void or_fmul(const void *a, const void *b, void *out);
void or_finv(const void *a, void *out);
void or_fexp(const void *a, const void *e /*u128 LE*/, void *out);
void or_root_of_unity(uint32_t log_n, void *out);
/* quadratic extension E = F[X]/(X^2 - X - 1): 32-byte values a || b (ext.h) */
void or_e2_mul(const void *x, const void *y, void *out);
void or_e2_inv(const void *x, void *out);

/* ---- NTT over f128 ---- */
/* evaluate polynomial (m coeffs) over offset * <w_size>, natural order */
int or_eval_coset(const void *coeffs, size_t m, size_t size, const void *offset, void *out);
/* interpolate `size` evaluations over offset * <w_size> into coefficients, in place */
int or_interp_coset(void *vals, size_t size, const void *offset);

/* ---- BLAKE3-256 (blake3 1.5.4, Cargo.lock:48) ---- */
void or_blake3(const uint8_t *in, size_t len, uint8_t out[32]);
void or_blake3_merge(const uint8_t l[32], const uint8_t r[32], uint8_t out[32]);
void or_merkle_root(const uint8_t *leaves, size_t num_leaves, uint8_t root[32]);

/* ---- Rescue (crypto/src/rescue.rs) ---- */
void or_rescue_apply_round(void *state4, uint8_t op_code, uint8_t op_value, uint64_t step);
void or_rescue_ark(uint32_t row, uint32_t col, void *out);

/* ---- VM front-end and trace generation (vm/src/program, vm/src/processor) ---- */
/* Program::compile.  codes/values get the padded op list; msg gets the reference error text. */
int or_program_compile(const char *source, uint8_t *codes, uint8_t *values, size_t cap, size_t *len,
                       void *hash_out /* 2 x 16 B */, char *msg, size_t msg_cap);
/* Processor::run + output + trace.  trace_out is 28 x n column-major (n <= cap_rows).
 * secret: num_secret ciphertexts of lwe_size elements each.  last_row: the 28 values the
 * reference draws from thread_rng() (vm/src/processor/mod.rs:86-92), supplied by the caller. */
int or_processor_trace(const uint8_t *codes, const uint8_t *values, size_t num_ops,
                       const uint8_t *public_in, size_t num_public,
                       const void *secret, size_t num_secret, uint32_t lwe_size, uint32_t delta,
                       const void *last_row, void *trace_out, size_t cap_rows, size_t *n_out,
                       void *outputs /* 16 x 16 B */, char *msg, size_t msg_cap);

/* ---- AIR (air/src/lib.rs:104-168) ---- */
void or_air_periodic_row(uint32_t step16, void *out9);
void or_air_eval_transition(const void *cur, const void *nxt, const void *periodic9,
                            uint32_t lwe_size, uint32_t delta, void *out20);

/* ---- full prove (winterfell 0.9 generate_proof restated; PARITY UNPINNED) ---- */
int or_prove(const void *trace /* 28 x n col-major */, size_t n, const or_options *opt,
             const or_pub_inputs *pub, uint8_t *proof_out, size_t *proof_len, or_record *rec,
             const or_dump *dump);

/* ---- verifier (winterfell verify restated for this AIR; checks our own proofs) ---- */
int or_verify(const uint8_t *proof, size_t proof_len, const or_pub_inputs *pub, uint32_t min_security,
              char *msg, size_t msg_cap);

#ifdef __cplusplus
}
#endif
#endif
