"""(debug) sharded loopback proofs in the normal and the measurement mode against the single-GPU proof."""
import hashlib, sys
sys.path[:0] = ["/root/repo", "/root/repo/encrypt-zkvm_amd", "/root/repo/tests"]
from zkvm_amd.prover import GpuProver, HostTrace, Program, ProofOptions, make_pub_inputs, vm_trace
from zkvm_amd.sharded import ShardedProver
from zkvm_amd.workloads import make_workload, ops_for_trace_len
log_n = int(sys.argv[1])
src = ops_for_trace_len(log_n, "cipher")
w = make_workload(src, seed=1000)
trace, outputs, h = vm_trace(src, w.public, w.secret, w.server_key, w.last_row)
n = trace.shape[1]
pub = make_pub_inputs(h, outputs, w.server_key.lwe_size(), w.server_key.parameters.delta)
host = HostTrace(n); host.array[...] = trace
prog = Program(src); inp = Program.encode_inputs(w.public, w.secret, w.server_key)
H = lambda b: hashlib.sha256(b).hexdigest()[:12]
g = GpuProver(0, max_trace_len=n)
want = H(g.prove_host(trace, pub, ProofOptions())[0])
g.close()
print("single", want, flush=True)
for G in (2, 4, 8):
    sp = ShardedProver.loopback(G, max_trace_len=n)
    sp.upload_trace(trace)
    for meas in (False, True):
        sp.set_measure(meas)
        sp.upload_trace(trace)  # (the vm proofs leave only their dynamic columns in the trace buffers)
        for kind, fn in (("device", lambda: sp.prove(None, pub, ProofOptions(), n=n)[0]),
                         ("host", lambda: sp.prove(host.array, pub, ProofOptions())[0]),
                         ("vm", lambda: sp.prove_program(prog, inp, w.last_row)[2])):
            got = []
            for _ in range(3):
                try:
                    got.append(H(fn()))
                except Exception as e:
                    got.append(f"ERR {str(e)[:60]}")
            print(G, "measure" if meas else "normal", kind, "OK" if got == [want] * 3 else got, flush=True)
    sp.close()
