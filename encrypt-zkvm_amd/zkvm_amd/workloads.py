"""Synthetic, seeded workloads for the prove path (harness side, not the hot path).

The reference draws its randomness from `rand::thread_rng()` in three places:
  * ServerKey::new key bits and ServerKey::encrypt masks/noise (fhe/src/server_key.rs:20-62),
  * the last trace row (vm/src/processor/mod.rs:86-92).
Here every one of them comes from a seeded numpy Generator so traces (and proofs) are
reproducible.  The LWE restatement follows fhe/src/server_key.rs:41-76 exactly; with the example
parameters (p=8, q=128, k=4, std=2.41e-5) the rounded noise is always 0.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

P = 2**128 - 45 * 2**40 + 1


def rand_field(rng: np.random.Generator, lo: int = 0) -> int:
    while True:
        v = int.from_bytes(rng.bytes(16), "little")
        if lo <= v < P:
            return v


@dataclass
class LweParameters:
    """fhe/src/parameters.rs:13-21"""
    plaintext_modulus: int = 8
    ciphertext_modulus: int = 128
    k: int = 4
    std: float = 2.412390240121573e-05

    @property
    def delta(self) -> int:
        return self.ciphertext_modulus // self.plaintext_modulus


@dataclass
class ServerKey:
    """fhe/src/server_key.rs:14-76 (seeded)."""
    parameters: LweParameters = field(default_factory=LweParameters)
    seed: int = 0

    def __post_init__(self):
        self.rng = np.random.default_rng(self.seed)
        self.key = [int(self.rng.integers(0, 2)) for _ in range(self.parameters.k)]

    def lwe_size(self) -> int:
        return self.parameters.k + 1

    def encrypt(self, value: int) -> list[int]:
        mask = [rand_field(self.rng) for _ in range(self.parameters.k)]
        noise = float(self.rng.normal(0.0, self.parameters.std))
        scaled = int(round(abs(noise)))
        body = sum(m * s for m, s in zip(mask, self.key)) % P
        body = (body + self.parameters.delta * value) % P
        body = (body + scaled) % P if noise > 0 else (body - scaled) % P
        return mask + [body]

    def decrypt(self, ct: list[int]) -> int:
        applied = sum(c * s for c, s in zip(ct[: self.parameters.k], self.key)) % P
        m = (ct[self.parameters.k] - applied) % P
        log2_delta = int(np.log2(self.parameters.delta))
        round_bit = (m >> (log2_delta - 1)) & 1
        return ((m >> log2_delta) + round_bit) & 0xFF


LR_PROGRAM = """# linear regression (examples/linear_regression/lr.txt)
read2
read
smul
read2
read
smul
add2
read2
read
smul
add2
read2
read
smul
add2
read
sadd
"""


def push_add_program(k: int) -> str:
    """configs[1]: push.1 + k x (push.1, add)  -> 8 padded slots per pair."""
    return "\n".join(["push.1"] + ["push.1\nadd"] * k) + "\n"


def cipher_mix_program(blocks: int) -> tuple[str, int, int]:
    """configs[2]: READ2/ADD2/SMUL ciphertext mix.  Stack depth stays <= 11.

    read2 read smul ; blocks x (read2 read smul add2 push.3 push.5 mul add read sadd) ; ...
    Returns (source, #public inputs, #secret inputs).
    """
    lines = ["read2", "read", "smul"]
    n_pub, n_sec = 1, 1
    for _ in range(blocks):
        lines += ["read2", "read", "smul", "add2", "read", "sadd", "push.3", "push.5", "mul", "add", "read",
                  "smul"]
        n_pub += 3
        n_sec += 1
    # fold the scalar left by the last "add" back: stack = [scalar?]; keep the program valid
    return "\n".join(lines) + "\n", n_pub, n_sec


def padded_length(source: str) -> int:
    """Length of Program::compile's padded op list (vm/src/program/mod.rs:65-86), without hashing."""
    n = 0
    for line in source.splitlines():
        tok = line.split("#")[0].strip()
        if not tok:
            continue
        if tok.startswith("push"):
            n += (8 - n % 8) % 8
        if n % 16 >= 14:
            n += 16 - n % 16
        n += 1
    return n + (16 - n % 16)


def trace_length(source: str) -> int:
    """Processor::trace length: capacity = smallest 16*2^k > padded ops; n = next_pow2(capacity + 1)."""
    p = padded_length(source)
    cap = 16
    while cap <= p:
        cap *= 2
    return 2 * cap


def ops_for_trace_len(log_n: int, kind: str = "cipher") -> str:
    """A program whose trace is exactly 2^log_n rows, with its padded length ~3/4 of the capacity."""
    cap = 2 ** (log_n - 1)
    make = (lambda k: push_add_program(k)) if kind == "pushadd" else (lambda k: cipher_mix_program(k)[0])
    per = (padded_length(make(65)) - padded_length(make(1))) // 64
    k = max(1, (cap * 3 // 4) // per)
    src = make(k)
    assert trace_length(src) == 2 ** log_n, (log_n, k, padded_length(src))
    return src


@dataclass
class Workload:
    source: str
    public: list[int]
    secret: list[list[int]]
    server_key: ServerKey
    last_row: list[int]


def make_workload(source: str, seed: int = 1, n_pub: int | None = None, n_sec: int | None = None,
                  params: LweParameters | None = None) -> Workload:
    """Inputs for `source`: public u8 values for READ, ciphertexts for READ2 under a seeded ServerKey
    (params: its LWE parameters, default LweParameters(): lwe_size 5), and a random non-zero last row."""
    rng = np.random.default_rng(seed + 1000)
    sk = ServerKey(params, seed=seed) if params is not None else ServerKey(seed=seed)
    ops = [ln.split("#")[0].strip() for ln in source.splitlines()]
    ops = [o for o in ops if o]
    n_pub = n_pub if n_pub is not None else sum(o == "read" for o in ops)
    n_sec = n_sec if n_sec is not None else sum(o == "read2" for o in ops)
    public = [int(rng.integers(0, 8)) for _ in range(n_pub)]
    secret = [sk.encrypt(int(rng.integers(0, 8))) for _ in range(n_sec)]
    last_row = [rand_field(rng, lo=1) for _ in range(28)]
    return Workload(source, public, secret, sk, last_row)
