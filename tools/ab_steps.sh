#!/bin/bash
# bench ms/proof versus the timed step count (pipeline fill/drain share), one box
set -eo pipefail
O=gpurun_out; mkdir -p $O
for s in 20 100 20 100; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-verify --steps $s > $O/steps_$s.json 2>/dev/null
  python3 -c "import json,sys; d=json.loads(open('$O/steps_$s.json').read().strip().splitlines()[-1]); print('steps $s', d['ms_per_step'], 'dev', d['device_resident_ms'], 'lat', d['latency_ms'])"
done
