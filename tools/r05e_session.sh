#!/bin/bash
# Round-5 session e: the GPU suite on the current tree (two-part narrow upload first, coalesced row hashing), then
# A/B of the row hashing (ZK_HASH_CO=0: the round-4 kernels) on the bench workload and the single-call latency.
set -eo pipefail
O=gpurun_out
mkdir -p "$O"
if [ "${1:-tests}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread \
    > "$O/gpu_tests_r05e.log" 2>&1 || { tail -60 "$O/gpu_tests_r05e.log"; exit 1; }
  tail -1 "$O/gpu_tests_r05e.log"
fi
AB="--no-cpu-baseline --no-verify --ab --sharded-log-n 0"
for rep in 1 2 3; do
  for v in "co:" "old:ZK_HASH_CO=0"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 300 python3 bench.py $AB > "$O/hab_${name}_$rep.json" 2>> "$O/hab.err"
    python3 - "$name" "$O/hab_${name}_$rep.json" <<'PY'
import json, sys
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = b["kernel_ms"]
print(f"{sys.argv[1]:>4} {b['ms_per_step']:8.3f} ms  latency {b['latency_ms']}  steady {b['steady_state_ms']}  device "
      f"{b['device_resident_ms']}  hash_rows {k.get('hash_rows')}  ntt1 {k.get('ntt_pass1')} ntt2 {k.get('ntt_pass2')}")
PY
    echo -n "$name lat " && env $envs timeout -k 10 200 python3 tools/latency_ab.py 31 2>> "$O/hab.err"
  done
done | tee "$O/hash_ab.txt"
