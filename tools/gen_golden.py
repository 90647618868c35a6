"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

The reference's own tests pin nothing at the winterfell layer, so these
fixtures are produced by this repo's oracle (oracle/, a C restatement of the reference path)
and freeze its outputs: the GPU prover and any later refactor of the oracle must keep
reproducing them byte for byte.  Each case stores the VM inputs (source, public u8 inputs,
secret ciphertexts, the seeded last row), the resulting trace (.npy, uint64 (28, n, 2)), the
stage-wise transcript values (roots, z, FRI roots, positions, nonce) and the proof bytes.

    python tools/gen_golden.py          # rewrites tests/golden/
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "encrypt-zkvm_amd"):
    sys.path.insert(0, str(p))

from oracle import oracle as orc  # noqa: E402
from zkvm_amd.workloads import LR_PROGRAM, cipher_mix_program, make_workload, push_add_program  # noqa: E402

OUT = ROOT / "tests" / "golden"
P = 2**128 - 45 * 2**40 + 1

CASES = [
    # name, source, seed, option overrides
    ("lr", LR_PROGRAM, 1, {}),
    ("lr_grind10_q28", LR_PROGRAM, 5, {"grinding": 10, "num_queries": 28}),
    ("pushadd12", push_add_program(12), 2, {}),
    ("cipher8_b16_f4", cipher_mix_program(8)[0], 3, {"blowup": 16, "fri_folding": 4, "fri_rem_max_deg": 31}),
    ("cipher20", cipher_mix_program(20)[0], 4, {"num_queries": 40}),
    ("pushadd12_f2_r7", push_add_program(12), 6, {"fri_folding": 2, "fri_rem_max_deg": 7, "num_queries": 50}),
    ("lr_f16_r15", LR_PROGRAM, 7, {"fri_folding": 16, "fri_rem_max_deg": 15, "blowup": 32}),
    # FieldExtension::Quadratic: E-valued coefficients, OOD, DEEP, FRI
    ("lr_quad", LR_PROGRAM, 8, {"field_extension": 2}),
    ("pushadd12_quad_q43_f4", push_add_program(12), 9,
     {"field_extension": 2, "num_queries": 43, "fri_folding": 4, "fri_rem_max_deg": 31}),
    ("cipher8_quad_f2_g9", cipher_mix_program(8)[0], 10,
     {"field_extension": 2, "fri_folding": 2, "fri_rem_max_deg": 7, "grinding": 9}),
]


def hexs(values):
    return [f"{v:032x}" for v in values]


def rec_bytes(arr, count, width=16):
    raw = bytes(arr)
    return [raw[i * width:(i + 1) * width] for i in range(count)]


def main():
    orc.build()
    OUT.mkdir(parents=True, exist_ok=True)
    cases = []
    for name, src, seed, over in CASES:
        w = make_workload(src, seed=seed)
        codes, values, h = orc.program_compile(src)
        trace, outputs = orc.processor_trace(codes, values, w.public, w.secret, w.server_key.lwe_size(),
                                             w.server_key.parameters.delta, w.last_row)
        n = trace.shape[1]
        opts = orc.default_options(**over)
        pub = orc.make_pub(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
        proof, rec, _ = orc.prove(trace, pub, opts)
        assert orc.verify(proof, pub, 0)[0] == 0, name
        np.save(OUT / f"{name}.trace.npy", trace, allow_pickle=False)
        (OUT / f"{name}.proof").write_bytes(proof)
        fri = [bytes(rec.fri_roots[i]).hex() for i in range(rec.num_fri_layers)]
        cases.append({
            "name": name, "source": src, "seed": seed, "options": {f: getattr(opts, f) for f, _ in orc.Options._fields_},
            "public": list(w.public), "secret": [hexs(ct) for ct in w.secret], "last_row": hexs(w.last_row),
            "lwe_size": w.server_key.lwe_size(), "delta": w.server_key.parameters.delta,
            "trace_len": n, "program_hash": hexs(h), "stack_outputs": hexs(outputs),
            "trace_sha256": hashlib.sha256(trace.tobytes()).hexdigest(),
            "trace_root": bytes(rec.trace_root).hex(), "constraint_root": bytes(rec.constraint_root).hex(),
            "z": bytes(rec.z).hex(), "fri_roots": fri, "remainder_len": rec.remainder_len,
            "pow_nonce": rec.pow_nonce, "positions": [rec.positions[i] for i in range(rec.num_positions)],
            "proof_len": len(proof), "proof_sha256": hashlib.sha256(proof).hexdigest(),
        })
        print(f"{name}: n={n} proof={len(proof)} B nonce={rec.pow_nonce}")

    # primitive vectors: field ops, roots of unity, BLAKE3 of elements, a small coset NTT
    rnd = np.random.default_rng(9)
    xs = [int.from_bytes(rnd.bytes(16), "little") % P for _ in range(16)] + [0, 1, P - 1, 2**64, 2**127]
    ys = list(reversed(xs))
    prim = {
        "a": hexs(xs), "b": hexs(ys),
        "mul": hexs([orc.fop("or_fmul", a, b) for a, b in zip(xs, ys)]),
        "add": hexs([orc.fop("or_fadd", a, b) for a, b in zip(xs, ys)]),
        "sub": hexs([orc.fop("or_fsub", a, b) for a, b in zip(xs, ys)]),
        "inv": hexs([orc.fop("or_finv", a) for a in xs if a]),
        "roots": {str(k): f"{orc.root_of_unity(k):032x}" for k in (1, 2, 3, 8, 16, 20, 23, 40)},
        "blake3_elems": [orc.blake3(orc.to_bytes(xs[:k])).hex() for k in (1, 2, 4, 7, 8, 16, 21)],
        "coset_lde_in": hexs(xs[:16]),
        "coset_lde_out": hexs(orc.eval_coset(xs[:16], 128, 3)),
    }
    (OUT / "cases.json").write_text(json.dumps({"generator": "tools/gen_golden.py (oracle/ CPU restatement)",
                                                "cases": cases, "primitives": prim}, indent=1) + "\n")


if __name__ == "__main__":
    main()
