#!/bin/bash
# 2^22 host-resident throughput against the number of provers in flight (one box).
set -eo pipefail
O=gpurun_out
mkdir -p "$O"
for P in 2 3 4; do
  timeout -k 10 300 python3 bench.py --log-n 22 --steps 8 --warmup 2 --inflight $P --no-cpu-baseline --no-verify > "$O/inf22_$P.json" 2> "$O/inf22_$P.err"
  python3 -c "import json;d=json.load(open('$O/inf22_$P.json'));print('inflight $P', d['ms_per_step'], 'device', d['device_resident_ms'], 'latency', d['latency_ms'])"
done
