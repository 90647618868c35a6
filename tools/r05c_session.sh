#!/bin/bash
# Round-5 session c: the GPU suite on the current tree (rank-local fill tables of rank-sized provers), then the
# single-call latency A/B of the upload order (round-5 experiment knobs ZK_UPLOAD_FIRST / ZK_NARROW_FIRST).
set -eo pipefail
TAG=${1:-r05c}
O=gpurun_out
mkdir -p "$O"
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread \
    > "$O/gpu_tests_$TAG.log" 2>&1 || { tail -60 "$O/gpu_tests_$TAG.log"; exit 1; }
  tail -1 "$O/gpu_tests_$TAG.log"
fi
AB="--no-cpu-baseline --no-verify --ab --sharded-log-n 0"
for rep in 1 2; do
  for v in "base:" "f2:ZK_UPLOAD_FIRST=2" "f1:ZK_UPLOAD_FIRST=1" "nf:ZK_NARROW_FIRST=1" "nf2:ZK_NARROW_FIRST=1 ZK_UPLOAD_FIRST=2"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 300 python3 bench.py $AB > "$O/lat_${name}_$rep.json" 2>> "$O/lat_ab_$TAG.err"
    python3 - "$name" "$O/lat_${name}_$rep.json" <<'PY'
import json, sys
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>5} {b['ms_per_step']:8.3f} ms  latency {b['latency_ms']}  steady {b['steady_state_ms']}  device {b['device_resident_ms']}  vm {b['vm']['vm_prove_ms']}")
PY
  done
done | tee "$O/lat_ab_$TAG.txt"
