"""Full-size golden pins (BASELINE.json configs[2], [3], [4]) from the CPU oracle.

The small fixtures (tools/gen_golden.py) store whole traces and proofs; at 2^20 and 2^22 a trace is
448 MiB / 1.8 GiB, so these cases store only what regenerates and pins it: the workload recipe
(generator, log2 trace length, seed), the sha256 of the oracle VM's trace, the transcript values
(trace and constraint roots, z, FRI roots, positions, nonce) and the proof bytes (small).  The GPU tests
regenerate the trace with the product VM, require its sha256, prove on the GPU and require the proof's
sha256 to equal the oracle's (tests/test_gpu_parity.py::test_full_size_golden, test_sharded.py).

    python tools/gen_golden_large.py [name ...]     # ~100 s (2^20), ~150 s (2^20 quadratic), ~8 min (2^22), ~4 min (2^21)
"""
from __future__ import annotations

import hashlib
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "encrypt-zkvm_amd"):
    sys.path.insert(0, str(p))

from oracle import oracle as orc  # noqa: E402
from zkvm_amd.workloads import make_workload, ops_for_trace_len  # noqa: E402

OUT = ROOT / "tests" / "golden" / "large"

# name, log2 n, generator, workload seed, option overrides, BASELINE config
CASES = [
    ("c2_cipher_2p20", 20, "cipher", 1000, {}, "configs[2]"),
    ("c4_cipher_2p20_quad", 20, "cipher", 1000, {"num_queries": 43, "field_extension": 2}, "configs[4]"),
    ("c3_cipher_2p22", 22, "cipher", 1000, {}, "configs[3]"),
    # not a BASELINE config: the odd four-step split (pass-1 lines of 2^11 with a trailing radix-2 stage, pass-2
    # lines of 2^10) at full scale
    ("x_cipher_2p21", 21, "cipher", 2100, {}, "odd split 2^21"),
]


def main(names):
    orc.build()
    OUT.mkdir(parents=True, exist_ok=True)
    idx_path = OUT / "cases.json"
    index = json.loads(idx_path.read_text())["cases"] if idx_path.exists() else []
    index = {c["name"]: c for c in index}
    for name, log_n, kind, seed, over, cfg in CASES:
        if names and name not in names:
            continue
        src = ops_for_trace_len(log_n, kind)
        w = make_workload(src, seed=seed)
        t0 = time.perf_counter()
        codes, values, h = orc.program_compile(src)
        trace, outputs = orc.processor_trace(codes, values, w.public, w.secret, w.server_key.lwe_size(),
                                             w.server_key.parameters.delta, w.last_row)
        t_vm = time.perf_counter() - t0
        n = trace.shape[1]
        assert n == 1 << log_n
        opts = orc.default_options(**over)
        pub = orc.make_pub(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
        t0 = time.perf_counter()
        proof, rec, _ = orc.prove(trace, pub, opts)
        t_prove = time.perf_counter() - t0
        min_sec = 128 if over.get("field_extension") == 2 else 95
        assert orc.verify(proof, pub, min_sec)[0] == 0, name
        (OUT / f"{name}.proof").write_bytes(proof)
        index[name] = {
            "name": name, "baseline_config": cfg, "log_n": log_n, "generator": kind, "seed": seed,
            "options": {f: getattr(opts, f) for f, _ in orc.Options._fields_}, "min_security": min_sec,
            "program_hash": [f"{v:032x}" for v in h], "stack_outputs": [f"{v:032x}" for v in outputs],
            "trace_sha256": hashlib.sha256(trace.tobytes()).hexdigest(),
            "trace_root": bytes(rec.trace_root).hex(), "constraint_root": bytes(rec.constraint_root).hex(),
            "z": bytes(rec.z).hex(), "fri_roots": [bytes(rec.fri_roots[i]).hex() for i in range(rec.num_fri_layers)],
            "pow_nonce": rec.pow_nonce, "positions": [rec.positions[i] for i in range(rec.num_positions)],
            "proof_len": len(proof), "proof_sha256": hashlib.sha256(proof).hexdigest(),
            "oracle_seconds": {"vm": round(t_vm, 1), "prove": round(t_prove, 1)},
        }
        print(f"{name}: n=2^{log_n} proof={len(proof)} B vm {t_vm:.1f} s prove {t_prove:.1f} s", flush=True)
        del trace
        idx_path.write_text(json.dumps({"generator": "tools/gen_golden_large.py (oracle/ CPU restatement)",
                                        "cases": [index[k] for k in sorted(index)]}, indent=1) + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])
