#!/bin/bash
# Round-5 session n: provers in flight per GPU (2 / 3 / 4) on the final upload path, two rounds.
set -eo pipefail
O=gpurun_out
mkdir -p "$O"
AB="--no-cpu-baseline --ab --no-verify --sharded-log-n 0 --steps 30"
: > "$O/r05n_inflight_ab.txt"
for k in 1 2; do
  for P in 3 2 4; do
    timeout -k 10 300 python3 bench.py $AB --inflight $P > "$O/r05n_ab_p${P}_$k.json" 2>> "$O/r05n_ab.err"
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d.get('latency_ms'), d.get('device_resident_ms'), d.get('steady_state_ms'))" \
      "$O/r05n_ab_p${P}_$k.json" "P=$P $k" >> "$O/r05n_inflight_ab.txt"
  done
done
cat "$O/r05n_inflight_ab.txt"
