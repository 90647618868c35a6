#!/bin/bash
# provers in flight A/B on the default workload (alternating runs, one box): bash tools/ab_inflight.sh [P ...]
set -eo pipefail
mkdir -p gpurun_out
PS=${*:-2 3 4}
for i in 1 2; do
  for P in $PS; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify --ab --steps 20 --inflight $P > gpurun_out/abif_$P.json 2> gpurun_out/abif_$P.err
    python3 -c "import json,sys; b=json.loads(open('gpurun_out/abif_$P.json').read().strip().splitlines()[-1]); print('inflight $P', b['ms_per_step'], 'steady', b['steady_state_ms'], 'latency', b['latency_ms'], 'device', b['device_resident_ms'])"
  done
done
