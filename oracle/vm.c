/*
 * vm.c -- oracle: Rescue sponge, assembler and trace generator of the reference VM.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 *   Rescue128 / apply_round ............ crypto/src/rescue.rs:30-118
 *   Program::compile / padding ......... vm/src/program/mod.rs:37-131, parsers.rs:4-66
 *   Processor::run / trace / output .... vm/src/processor/mod.rs:61-118
 *   Stack / Decoder / System / Chiplets  vm/src/processor/{stack,decoder,system,chiplets}.rs
 *   ServerKey add / scalar_add / scalar_mul  fhe/src/server_key.rs:78-124
 */
#include <stdio.h>

#include "internal.h"
#include "rescue_consts.h"

#define CYCLE 16
#define NUM_ROUNDS 14
#define INV_ALPHA (((u128)0xaaaaaaaaaaaaaaaaULL << 64) | 0xaaaa8caaaaaaaaabULL)

static u128 ark_u(unsigned r, unsigned c) { return ((u128)OR_ARK[8 * r + c][1] << 64) | OR_ARK[8 * r + c][0]; }
static u128 mds_u(const uint64_t m[16][2], unsigned i) { return ((u128)m[i][1] << 64) | m[i][0]; }

void or_rescue_ark(uint32_t row, uint32_t col, void *out) { st(out, ark_u(row % 16, col % 8)); }

static void apply_mds_u(u128 *s, const uint64_t m[16][2]) {
    u128 r[4];
    for (int i = 0; i < 4; i++) {
        r[i] = 0;
        for (int j = 0; j < 4; j++) r[i] = f_add(r[i], f_mul(mds_u(m, 4 * i + j), s[j]));
    }
    memcpy(s, r, sizeof r);
}

/* crypto/src/rescue.rs:102-118 */
static void apply_round_u(u128 *s, uint8_t op_code, uint8_t op_value, uint64_t step) {
    unsigned r = (unsigned)(step % CYCLE);
    for (int i = 0; i < 4; i++) s[i] = f_exp(s[i], 3);
    apply_mds_u(s, OR_MDS);
    for (int i = 0; i < 4; i++) s[i] = f_add(s[i], ark_u(r, i));
    s[0] = f_add(s[0], op_code);
    s[1] = f_add(s[1], op_value);
    for (int i = 0; i < 4; i++) s[i] = f_exp(s[i], INV_ALPHA);
    apply_mds_u(s, OR_MDS);
    for (int i = 0; i < 4; i++) s[i] = f_add(s[i], ark_u(r, 4 + i));
}

void or_rescue_apply_round(void *state4, uint8_t op_code, uint8_t op_value, uint64_t step) {
    u128 s[4];
    memcpy(s, state4, 64);
    apply_round_u(s, op_code, op_value, step);
    memcpy(state4, s, 64);
}

/* Rescue128::update, rescue.rs:46-56 */
static void sponge_update(u128 *s, uint64_t *step, uint8_t code, uint8_t value) {
    if (*step % CYCLE < NUM_ROUNDS)
        apply_round_u(s, code, value, *step);
    else
        s[2] = s[3] = 0;
    (*step)++;
}

/* ---------------------------------------------------------------- assembler */
enum { OP_NOOP = 0x00, OP_PUSH = 0x10, OP_READ = 0x11, OP_READ2 = 0x12, OP_ADD = 0x08, OP_MUL = 0x09,
       OP_SADD = 0x0a, OP_SMUL = 0x0c, OP_ADD2 = 0x0b };

static const char *op_name(uint8_t c) {
    switch (c) {
    case OP_NOOP: return "noop";
    case OP_PUSH: return "push";
    case OP_READ: return "read";
    case OP_READ2: return "read2";
    case OP_ADD: return "add";
    case OP_MUL: return "mul";
    case OP_SADD: return "sadd";
    case OP_SMUL: return "smul";
    case OP_ADD2: return "add2";
    }
    return "?";
}

static void op_display(uint8_t c, uint8_t v, char *buf, size_t cap) {
    if (c == OP_PUSH)
        snprintf(buf, cap, "push(%u)", v);
    else
        snprintf(buf, cap, "%s", op_name(c));
}

static char *trim(char *s) {
    while (*s == ' ' || *s == '\t' || *s == '\r') s++;
    size_t n = strlen(s);
    while (n && (s[n - 1] == ' ' || s[n - 1] == '\t' || s[n - 1] == '\r')) s[--n] = 0;
    return s;
}

static size_t pad16(size_t len) { return len + (CYCLE - len % CYCLE); } /* compute_padding, mod.rs:124 */

/* parse one token "name[.param...]" -> code/value; mirrors parse_op + parsers.rs */
static int parse_op(size_t step, const char *tok, uint8_t *code, uint8_t *value, char *msg, size_t cap) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s", tok);
    char *parts[64];
    int np = 0;
    char *p = buf;
    parts[np++] = p;
    for (; *p; p++)
        if (*p == '.' && np < 64) {
            *p = 0;
            parts[np++] = p + 1;
        }
    const char *name = parts[0];
    static const struct { const char *n; uint8_t c; } tab[] = {
        {"push", OP_PUSH}, {"read", OP_READ}, {"read2", OP_READ2}, {"add", OP_ADD},
        {"mul", OP_MUL}, {"sadd", OP_SADD}, {"smul", OP_SMUL}, {"add2", OP_ADD2}};
    int found = -1;
    for (int i = 0; i < 8; i++)
        if (!strcmp(name, tab[i].n)) found = i;
    if (found < 0) {
        snprintf(msg, cap, "program error at %zu: instruction %s is invalid", step, tok);
        return OR_ERR_PROGRAM;
    }
    *code = tab[found].c;
    *value = 0;
    if (*code == OP_PUSH) {
        if (np == 1) {
            snprintf(msg, cap, "program error at %zu: malformed instruction push, parameter is missing", step);
            return OR_ERR_PROGRAM;
        }
        if (np > 2) {
            snprintf(msg, cap, "program error at %zu: malformed instruction push, too many parameters provided", step);
            return OR_ERR_PROGRAM;
        }
        /* u8::from_str: optional '+', decimal digits, value <= 255 */
        const char *d = parts[1];
        if (*d == '+') d++;
        int ok = *d != 0;
        unsigned long v = 0;
        for (const char *q = d; *q && ok; q++) {
            if (*q < '0' || *q > '9') ok = 0;
            else if ((v = v * 10 + (unsigned long)(*q - '0')) > 255) ok = 0;
        }
        if (!ok) {
            snprintf(msg, cap, "program error at %zu: malformed instruction push, parameter '%s' is invalid", step,
                     parts[1]);
            return OR_ERR_PROGRAM;
        }
        *value = (uint8_t)v;
    } else if (np > 1) {
        snprintf(msg, cap, "program error at %zu: malformed instruction %s, too many parameters provided", step, name);
        return OR_ERR_PROGRAM;
    }
    return OR_OK;
}

int or_program_compile(const char *source, uint8_t *codes, uint8_t *values, size_t cap, size_t *len, void *hash_out,
                       char *msg, size_t msg_cap) {
    char dummy[8];
    if (!msg) {
        msg = dummy;
        msg_cap = sizeof dummy;
    }
    msg[0] = 0;
    size_t srclen = strlen(source);
    char *src = (char *)malloc(srclen + 1);
    memcpy(src, source, srclen + 1);
    size_t ntok = 0, code_len = 0;
    int rc = OR_OK;
    /* tokenize by lines (str::lines), drop comments and blank lines (mod.rs:42-60) */
    char **toks = (char **)malloc(sizeof(char *) * (srclen / 2 + 2));
    for (char *line = src; line;) {
        char *nl = strchr(line, '\n');
        if (nl) *nl = 0;
        char *t = trim(line);
        if (*t && *t != '#') {
            char *h = strchr(t, '#');
            if (h) *h = 0;
            t = trim(t);
            if (*t) toks[ntok++] = t;
        }
        line = nl ? nl + 1 : NULL;
    }
    if (ntok == 0) {
        snprintf(msg, msg_cap, "program error at 0: a program must contain at least one instruction");
        rc = OR_ERR_PROGRAM;
        goto done;
    }
    for (size_t i = 0; i < ntok; i++) {
        uint8_t c, v;
        rc = parse_op(i + 1, toks[i], &c, &v, msg, msg_cap);
        if (rc) goto done;
        size_t target = code_len;
        if (c == OP_PUSH) target = code_len + (8 - code_len % 8) % 8; /* PUSH_OP_ALIGNMENT */
        if (target % CYCLE >= NUM_ROUNDS) target = pad16(target);
        if (target + 1 > cap) {
            rc = OR_ERR_BUFFER_TOO_SMALL;
            goto done;
        }
        for (; code_len < target; code_len++) codes[code_len] = values[code_len] = 0;
        codes[code_len] = c;
        values[code_len++] = v;
    }
    {
        size_t target = pad16(code_len);
        if (target > cap) {
            rc = OR_ERR_BUFFER_TOO_SMALL;
            goto done;
        }
        for (; code_len < target; code_len++) codes[code_len] = values[code_len] = 0;
    }
    {
        u128 s[4] = {0, 0, 0, 0};
        uint64_t step = 0;
        for (size_t i = 0; i < code_len; i++) sponge_update(s, &step, codes[i], values[i]);
        if (hash_out) {
            st((uint8_t *)hash_out, s[0]);
            st((uint8_t *)hash_out + 16, s[1]);
        }
    }
    *len = code_len;
done:
    free(toks);
    free(src);
    return rc;
}

/* ---------------------------------------------------------------- processor */
#define MAX_STACK 16

int or_processor_trace(const uint8_t *codes, const uint8_t *values, size_t num_ops, const uint8_t *public_in,
                       size_t num_public, const void *secret, size_t num_secret, uint32_t lwe_size, uint32_t delta,
                       const void *last_row, void *trace_out, size_t cap_rows, size_t *n_out, void *outputs,
                       char *msg, size_t msg_cap) {
    char dummy[8];
    if (!msg) {
        msg = dummy;
        msg_cap = sizeof dummy;
    }
    msg[0] = 0;
    if (lwe_size == 0 || lwe_size > 15) return OR_ERR_INVALID_ARG;
    /* all four state machines start at MIN_TRACE_LENGTH = 16 rows and double together */
    size_t capacity = 16;
    while (capacity <= num_ops) capacity *= 2;
    size_t rows = capacity; /* capacity of every component after num_ops steps */
    u128 *reg = (u128 *)calloc((size_t)MAX_STACK * rows, 16); /* reg[i*rows + clk] */
    u128 *helper = (u128 *)calloc(rows, 16);
    u128 *bits = (u128 *)calloc(5 * rows, 16);
    u128 *hflag = (u128 *)calloc(rows, 16);
    u128 *sponge = (u128 *)calloc(4 * rows, 16);
    const u128 *sec = (const u128 *)secret;
    size_t tape_a = 0, tape_b = 0, depth = 0, clk = 0;
    u128 s[4] = {0, 0, 0, 0};
    uint64_t sstep = 0;
    int rc = OR_OK;
    char opbuf[32];
#define R(i, c) reg[(size_t)(i) * rows + (c)]
    for (size_t k = 0; k < num_ops; k++) {
        uint8_t c = codes[k], v = values[k];
        clk++;
        op_display(c, v, opbuf, sizeof opbuf);
        /* ---- Stack::execute_op (stack.rs:48-70) */
        switch (c) {
        case OP_NOOP:
            for (size_t i = 0; i < depth; i++) R(i, clk) = R(i, clk - 1);
            break;
        case OP_PUSH:
        case OP_READ:
        case OP_READ2: {
            size_t cnt = c == OP_READ2 ? lwe_size : 1;
            /* op_read2 pops its input before shift_right; op_read shifts first (stack.rs:107-131) */
            if (c == OP_READ2 && tape_b >= num_secret) goto empty;
            depth += cnt;
            if (c == OP_READ && depth <= MAX_STACK && tape_a >= num_public) goto empty;
            if (depth > MAX_STACK) {
                snprintf(msg, msg_cap, "stack error at %zu: %s operation stack overflow", clk, opbuf);
                rc = OR_ERR_STACK;
                goto out;
            }
            for (size_t i = 0; i < depth - cnt; i++) R(i + cnt, clk) = R(i, clk - 1);
            if (c == OP_PUSH) R(0, clk) = v;
            else if (c == OP_READ) R(0, clk) = public_in[tape_a++];
            else {
                for (size_t i = 0; i < lwe_size; i++) R(i, clk) = sec[tape_b * lwe_size + i];
                tape_b++;
            }
            break;
        empty:
            snprintf(msg, msg_cap, "stack error at %zu: no more inputs to %s", clk, opbuf);
            rc = OR_ERR_STACK;
            goto out;
        }
        default: {
            size_t need = c == OP_ADD || c == OP_MUL ? 2 : c == OP_ADD2 ? 2 * lwe_size : lwe_size + 1;
            size_t start = need, pos = c == OP_ADD2 ? lwe_size : 1;
            if (depth < need) {
                snprintf(msg, msg_cap, "stack error at %zu: %s operation stack underflow", clk, opbuf);
                rc = OR_ERR_STACK;
                goto out;
            }
            if (c == OP_ADD) R(0, clk) = f_add(R(0, clk - 1), R(1, clk - 1));
            else if (c == OP_MUL) R(0, clk) = f_mul(R(0, clk - 1), R(1, clk - 1));
            else if (c == OP_SADD) {
                /* scalar_add: ct + encrypt_trivial(scalar) = ct + [0..0, delta*scalar] */
                for (size_t i = 0; i < lwe_size; i++) {
                    u128 t = R(1 + i, clk - 1);
                    if (i == lwe_size - 1) t = f_add(t, f_mul((u128)delta, R(0, clk - 1)));
                    R(i, clk) = t;
                }
            } else if (c == OP_SMUL) {
                for (size_t i = 0; i < lwe_size; i++) R(i, clk) = f_mul(R(1 + i, clk - 1), R(0, clk - 1));
            } else { /* ADD2 */
                for (size_t i = 0; i < lwe_size; i++) R(i, clk) = f_add(R(i, clk - 1), R(i + lwe_size, clk - 1));
            }
            /* shift_left(op, start, pos) */
            for (size_t i = start; i < depth; i++) R(i - pos, clk) = R(i, clk - 1);
            for (size_t i = depth - pos; i < depth; i++) R(i, clk) = 0;
            depth -= pos;
        }
        }
        helper[clk] = depth; /* set_helpers */
        /* ---- Decoder::decode_op (decoder.rs:49-76): row clk-1 holds bit i of the opcode */
        for (int i = 0; i < 5; i++) bits[(size_t)i * rows + clk - 1] = (c >> i) & 1;
        /* ---- Chiplets::hash_op (chiplets.rs:69-112) */
        if (!(sstep % CYCLE < NUM_ROUNDS) && c != OP_NOOP) {
            snprintf(msg, msg_cap, "chiplets error at %zu: expected noop but was %s", clk, opbuf);
            rc = OR_ERR_CHIPLETS;
            goto out;
        }
        sponge_update(s, &sstep, c, v);
        hflag[clk - 1] = 1;
        for (int i = 0; i < 4; i++) sponge[(size_t)i * rows + clk] = s[i];
    }
    if (clk % CYCLE != 0) {
        snprintf(msg, msg_cap, "chiplets error at %zu: trace length should be a multiple of %d, but was %zu", clk,
                 CYCLE, clk);
        rc = OR_ERR_CHIPLETS;
        goto out;
    }
    {
        /* Processor::trace (mod.rs:71-95): n = next_pow2(capacity + NUM_RAND_ROWS) */
        size_t n = 1;
        while (n < capacity + 1) n *= 2;
        if (n > cap_rows) {
            rc = OR_ERR_BUFFER_TOO_SMALL;
            *n_out = n;
            goto out;
        }
        u128 *t = (u128 *)trace_out;
        const u128 *last = (const u128 *)last_row;
        for (size_t r = 0; r < n; r++) {
            size_t rr = r <= clk ? r : clk; /* rows after the program repeat the final state */
            t[0 * n + r] = r;               /* System: clk column */
            for (int i = 0; i < 5; i++) t[(size_t)(1 + i) * n + r] = r <= clk ? bits[(size_t)i * rows + r] : 0;
            t[6 * n + r] = r <= clk ? hflag[r] : 0;
            for (int i = 0; i < 4; i++) t[(size_t)(7 + i) * n + r] = sponge[(size_t)i * rows + rr];
            t[11 * n + r] = helper[rr];
            for (int i = 0; i < MAX_STACK; i++) t[(size_t)(12 + i) * n + r] = R(i, rr);
        }
        for (int col = 0; col < 28; col++) t[(size_t)col * n + n - 1] = last[col];
        *n_out = n;
        if (outputs)
            for (int i = 0; i < MAX_STACK; i++) st((uint8_t *)outputs + 16 * i, R(i, clk));
    }
out:
#undef R
    free(reg);
    free(helper);
    free(bits);
    free(hflag);
    free(sponge);
    return rc;
}
