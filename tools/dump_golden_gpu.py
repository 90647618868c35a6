"""Prove every golden case on the GPU and write the proof bytes to gpurun_out/<case>.gpu.proof
(for byte-level diffing against tests/golden/<case>.proof on the host)."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "encrypt-zkvm_amd")]
from zkvm_amd.prover import GpuProver, ProofOptions, make_pub_inputs  # noqa: E402

G = ROOT / "tests" / "golden"
OUT = ROOT / "gpurun_out"
OUT.mkdir(exist_ok=True)
for c in json.loads((G / "cases.json").read_text())["cases"]:
    trace = np.load(G / f"{c['name']}.trace.npy", allow_pickle=False)
    o = c["options"]
    opts = ProofOptions(o["num_queries"], o["blowup"], o["grinding"], o["field_extension"], o["fri_folding"],
                        o["fri_rem_max_deg"])
    pub = make_pub_inputs([int(h, 16) for h in c["program_hash"]], [int(h, 16) for h in c["stack_outputs"]],
                          c["lwe_size"], c["delta"])
    g = GpuProver(0, max_trace_len=trace.shape[1], max_blowup=o["blowup"])
    proof, rec, _, rc = g.prove(trace, pub, opts, record=True, dump=("fri_layer1",))
    g.close()
    (OUT / f"{c['name']}.gpu.proof").write_bytes(proof)
    print(c["name"], rc, len(proof), proof == (G / f"{c['name']}.proof").read_bytes())
