"""Order-dependence probe: prove a sequence of (log_n, blowup, ext) cases in one process."""
import sys
sys.path.insert(0, "encrypt-zkvm_amd")
from zkvm_amd.prover import vm_trace, GpuProver, ProofOptions, make_pub_inputs
from zkvm_amd.workloads import make_workload, ops_for_trace_len
for spec in sys.argv[1:]:
    lg, bl, ext = (int(x) for x in spec.split(":"))
    src = ops_for_trace_len(lg, "cipher")
    w = make_workload(src, seed=21)
    trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
    pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
    g = GpuProver(0, max_trace_len=trace.shape[1], max_blowup=bl)
    try:
        r = g.prove(trace, pub, ProofOptions(field_extension=ext, blowup_factor=bl, num_queries=28 if bl == 16 else 32))
        print(spec, "rc", r[3], "len", len(r[0]), flush=True)
    except Exception as e:
        print(spec, "EXC", e, flush=True)
    finally:
        g.close()
