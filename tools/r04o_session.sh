#!/bin/bash
# device-side clock detection: full GPU suite, the bench line, the sharded loopback fit
set -o pipefail
O=gpurun_out
mkdir -p $O
bash tools/gpu_full_check.sh r04o || exit 1
python3 -c "import json;d=json.load(open('$O/bench_r04o.json'));print(d['ms_per_step'],d['latency_ms'],d['device_resident_ms'],d['steady_state_ms'],d['proof_matches_pin'],d['vm']['vm_prove_ms'])"
timeout -k 10 400 python3 tools/shard_model.py 22 3 > $O/shard_model_r04o.json 2> $O/shard_model_r04o.err || { tail -5 $O/shard_model_r04o.err; exit 1; }
cat $O/shard_model_r04o.err | tail -4
