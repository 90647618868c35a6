#!/bin/bash
# Round-5 session k: zk_vm_prove with the preprocessed columns' work queued before the host stack pass (ZK_VM_PREFIX):
# the vm GPU tests, one-call vm latency A/B (3 x 31 calls), the full GPU suite, the default bench line.
set -eo pipefail
O=gpurun_out
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_vm.py -m gpu -x -q --timeout 280 --timeout-method thread \
  > "$O/gpu_vm_tests_r05k.log" 2>&1 || { tail -60 "$O/gpu_vm_tests_r05k.log"; exit 1; }
tail -1 "$O/gpu_vm_tests_r05k.log"
: > "$O/r05k_vm_latency_ab.txt"
for k in 1 2 3; do
  for v in "off:ZK_VM_PREFIX=0" "on:"; do
    name=${v%%:*}; envs=${v#*:}
    echo -n "$name $k " >> "$O/r05k_vm_latency_ab.txt"
    timeout -k 10 180 env $envs python3 tools/vm_latency_ab.py 31 >> "$O/r05k_vm_latency_ab.txt"
  done
done
cat "$O/r05k_vm_latency_ab.txt"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread \
  > "$O/gpu_tests_r05k.log" 2>&1 || { tail -60 "$O/gpu_tests_r05k.log"; exit 1; }
tail -1 "$O/gpu_tests_r05k.log"
timeout -k 10 600 python3 bench.py > "$O/bench_r05k.json" 2> "$O/bench_r05k.err" || { tail -20 "$O/bench_r05k.err"; exit 1; }
cat "$O/bench_r05k.json"
