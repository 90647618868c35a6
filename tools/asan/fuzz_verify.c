/* fuzz_verify.c -- host-only fuzz driver for the untrusted-input parsers, built with AddressSanitizer and
 * UndefinedBehaviorSanitizer (make asan in encrypt-zkvm_amd/ and oracle/; run by tests/test_asan.py).
 *
 * Targets (one build each, selected by -DTARGET_PRODUCT or -DTARGET_ORACLE):
 *   product: zk_verify (encrypt-zkvm_amd/csrc/verifier.cpp) and zk_vm_trace (the assembler + VM, csrc/vm.cpp)
 *   oracle:  or_verify (oracle/verifier.c) and or_program_compile + or_processor_trace (oracle/vm.c)
 *
 * Usage: fuzz_verify <cases file> <seed> <flips per proof>
 *   cases file: lines "proof_path pub_path min_security" (pub: the 296-byte zk_pub_inputs / or_pub_inputs).
 * For every proof: the original must verify; every truncation (all lengths up to 4 KiB, then a stride) must
 * be rejected; <flips> random single-byte changes must be rejected; random garbage must be rejected.  Then the
 * assembler gets mutated program texts with random input vectors (any status is fine, nothing may fault).
 * Exit status 0 when every check holds; the sanitizers abort on the first memory or UB error.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define PUB_BYTES 296

#if defined(TARGET_PRODUCT)
#include "../../include/zkvm_gpu.h"
typedef zk_pub_inputs pub_t;
static int verify(const uint8_t *p, size_t n, const pub_t *pub, uint32_t sec) {
    char msg[256];
    return zk_verify(p, n, pub, sec, msg, sizeof msg);
}
static int assemble_and_run(const char *src, const uint8_t *pubin, size_t npub, const uint8_t *sec, size_t nsec,
                            const uint8_t *last_row) {
    size_t n = 0;
    uint8_t outputs[256], hash[32];
    int rc = zk_vm_trace(src, pubin, npub, sec, nsec, 5, 16, last_row, NULL, 0, &n, outputs, hash);
    if (rc != ZK_ERR_BUFFER_TOO_SMALL || n == 0 || n > (1u << 14)) return rc;
    uint8_t *trace = (uint8_t *)malloc(28 * n * 16);
    rc = zk_vm_trace(src, pubin, npub, sec, nsec, 5, 16, last_row, trace, n, &n, outputs, hash);
    free(trace);
    return rc;
}
#define NAME "product (zk_verify, zk_vm_trace)"
#elif defined(TARGET_ORACLE)
#include "../../oracle/oracle.h"
typedef or_pub_inputs pub_t;
static int verify(const uint8_t *p, size_t n, const pub_t *pub, uint32_t sec) {
    char msg[256];
    return or_verify(p, n, pub, sec, msg, sizeof msg);
}
static int assemble_and_run(const char *src, const uint8_t *pubin, size_t npub, const uint8_t *sec, size_t nsec,
                            const uint8_t *last_row) {
    static uint8_t codes[1 << 14], values[1 << 14];
    size_t len = 0;
    uint8_t hash[32];
    char msg[512];
    int rc = or_program_compile(src, codes, values, sizeof codes, &len, hash, msg, sizeof msg);
    if (rc) return rc;
    size_t cap = 16;
    while (cap <= len) cap *= 2;
    cap *= 2;
    if (cap > (1u << 14)) return 0;
    uint8_t *trace = (uint8_t *)malloc(28 * cap * 16);
    uint8_t outputs[256];
    size_t n = 0;
    rc = or_processor_trace(codes, values, len, pubin, npub, sec, nsec, 5, 16, last_row, trace, cap, &n, outputs, msg,
                            sizeof msg);
    free(trace);
    return rc;
}
#define NAME "oracle (or_verify, or_program_compile / or_processor_trace)"
#else
#error "build with -DTARGET_PRODUCT or -DTARGET_ORACLE"
#endif

static uint64_t rng_state;
static uint64_t rnd(void) {  /* splitmix64 */
    uint64_t z = (rng_state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static uint8_t *read_file(const char *path, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *b = (uint8_t *)malloc(n > 0 ? (size_t)n : 1);
    if (n > 0 && fread(b, 1, (size_t)n, f) != (size_t)n) {
        fclose(f);
        free(b);
        return NULL;
    }
    fclose(f);
    *len = (size_t)n;
    return b;
}

/* a copy in a buffer of exactly `len` bytes, so any read past the end is a heap overflow */
static int verify_exact(const uint8_t *p, size_t len, const pub_t *pub, uint32_t sec) {
    uint8_t *c = (uint8_t *)malloc(len ? len : 1);
    if (len) memcpy(c, p, len);
    int rc = verify(len ? c : NULL, len, pub, sec);
    free(c);
    return rc;
}

static const char *TOKENS[] = {"push.1", "push.0", "push.255", "push.256", "push.99999999999999999999999", "push.",
                               "push.-3", "push.x", "read", "read2", "add", "add2", "mul", "smul", "sadd", "noop",
                               "# comment", "", " ", "\t", "pop", "push.3 push.4", "READ", "read2read", "push.12",
                               "add ; add", "push.18446744073709551616", "\xff\xfe", "pus", "push.1\r"};

static void fuzz_assembler(int iters) {
    const int nt = (int)(sizeof TOKENS / sizeof TOKENS[0]);
    char *src = (char *)malloc(1 << 16);
    uint8_t pubin[64], last_row[28 * 16];
    uint8_t *sec = (uint8_t *)malloc(16 * 5 * 64);
    int ok = 0, err = 0;
    /* half the programs: blocks of the cipher-mix program (zkvm_amd/workloads.py) with a few token-level
     * mutations, so the VM runs far; the other half: arbitrary token soup, so the parser sees garbage */
    static const char *BLOCK[] = {"read2", "read", "smul", "add2", "read", "sadd", "push.3", "push.5", "mul", "add",
                                  "read", "smul"};
    const int nb = (int)(sizeof BLOCK / sizeof BLOCK[0]);
    for (int it = 0; it < iters; it++) {
        size_t pos = 0;
        const int structured = it & 1;
        const int lines = (int)(rnd() % 200);
        if (structured) {
            memcpy(src, "read2\nread\nsmul\n", 16);
            pos = 16;
        }
        for (int l = 0; l < lines && pos < (1 << 16) - 64; l++) {
            const char *t = structured ? (rnd() % 40 ? BLOCK[l % nb] : TOKENS[rnd() % nt]) : TOKENS[rnd() % nt];
            size_t k = strlen(t);
            memcpy(src + pos, t, k);
            pos += k;
            src[pos++] = (structured || rnd() % 17) ? '\n' : ' ';
        }
        if (!structured && rnd() % 5 == 0 && pos > 0) src[rnd() % pos] = (char)(rnd() & 0xff);  /* a random byte */
        if (!structured && rnd() % 7 == 0) pos = rnd() % (pos + 1);                            /* cut mid-token */
        src[pos] = 0;
        const size_t npub = structured ? 64 - rnd() % 4 : rnd() % 65, nsec = structured ? 64 - rnd() % 4 : rnd() % 65;
        for (size_t i = 0; i < npub; i++) pubin[i] = (uint8_t)rnd();
        for (size_t i = 0; i < 16 * 5 * nsec; i++) sec[i] = (uint8_t)rnd();
        for (size_t i = 0; i < 16 * 5 * nsec; i += 16) sec[i + 15] &= 0x7f;  /* mostly canonical elements */
        for (int i = 0; i < 28 * 16; i++) last_row[i] = (uint8_t)rnd();
        for (int i = 0; i < 28; i++) last_row[16 * i + 15] &= 0x7f;
        if (assemble_and_run(src, npub ? pubin : NULL, npub, nsec ? sec : NULL, nsec, last_row) == 0) ok++;
        else err++;
    }
    printf("  assembler: %d programs (%d ran, %d refused)\n", iters, ok, err);
    free(src);
    free(sec);
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s <cases file> <seed> <flips per proof>\n", argv[0]);
        return 64;
    }
    rng_state = strtoull(argv[2], NULL, 10);
    const int flips = atoi(argv[3]);
    FILE *cf = fopen(argv[1], "r");
    if (!cf) {
        fprintf(stderr, "cannot open %s\n", argv[1]);
        return 64;
    }
    printf("fuzz_verify: %s\n", NAME);
    char pp[1024], up[1024];
    unsigned sec;
    int failures = 0, cases = 0;
    long checks = 0;
    while (fscanf(cf, "%1023s %1023s %u", pp, up, &sec) == 3) {
        size_t plen = 0, ulen = 0;
        uint8_t *proof = read_file(pp, &plen), *pubb = read_file(up, &ulen);
        if (!proof || !pubb || ulen != PUB_BYTES) {
            fprintf(stderr, "bad case %s %s\n", pp, up);
            return 64;
        }
        pub_t pub;
        memcpy(&pub, pubb, sizeof pub);
        cases++;
        int accepted = 0;
        if (verify_exact(proof, plen, &pub, sec) != 0) {
            printf("  FAIL %s: the original proof is rejected\n", pp);
            failures++;
        }
        checks++;
        /* truncations */
        for (size_t L = 0; L < plen; L += (L < 4096 ? 1 : 97 + rnd() % 64)) {
            if (verify_exact(proof, L, &pub, sec) == 0) accepted++;
            checks++;
        }
        /* one extra trailing byte */
        uint8_t *longer = (uint8_t *)malloc(plen + 1);
        memcpy(longer, proof, plen);
        longer[plen] = 0;
        if (verify_exact(longer, plen + 1, &pub, sec) == 0) accepted++;
        free(longer);
        /* single-byte changes */
        uint8_t *m = (uint8_t *)malloc(plen);
        for (int f = 0; f < flips; f++) {
            memcpy(m, proof, plen);
            const size_t at = rnd() % plen;
            m[at] ^= (uint8_t)(1 + rnd() % 255);
            if (verify_exact(m, plen, &pub, sec) == 0) {
                accepted++;
                printf("  accepted a change at byte %zu of %s\n", at, pp);
            }
            checks++;
        }
        /* garbage of random lengths, and the proof with a random tail */
        for (int g = 0; g < 50; g++) {
            const size_t L = rnd() % (plen + 64);
            uint8_t *b = (uint8_t *)malloc(L ? L : 1);
            const size_t keep = g & 1 ? (L < plen ? L : plen) * (rnd() % 100) / 100 : 0;
            if (keep) memcpy(b, proof, keep);
            for (size_t i = keep; i < L; i++) b[i] = (uint8_t)rnd();
            if (verify_exact(b, L, &pub, sec) == 0) accepted++;
            free(b);
            checks++;
        }
        free(m);
        if (accepted) {
            printf("  FAIL %s: %d modified proofs accepted\n", pp, accepted);
            failures++;
        }
        free(proof);
        free(pubb);
    }
    fclose(cf);
    printf("  proofs: %d cases, %ld verifier calls\n", cases, checks);
    fuzz_assembler(400);
    printf("fuzz_verify: %s\n", failures ? "FAILED" : "ok");
    return failures ? 1 : 0;
}
