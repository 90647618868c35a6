#!/bin/bash
# A/B environment settings on the default bench workload, alternating runs:
#   bash tools/ab_env.sh "NAME=VAL ..." "NAME=VAL ..." ...   ("-" = no extra settings)
# Each entry: one bench line (no CPU baseline, no verification); prints ms_per_step.
set -eo pipefail
O=gpurun_out
mkdir -p "$O"
i=0
for v in "$@"; do
  i=$((i + 1))
  envs=()
  [ "$v" != "-" ] && read -r -a envs <<< "$v"
  env "${envs[@]}" timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} \
    > "$O/abenv_$i.json" 2> "$O/abenv_$i.err" || { echo "$v FAILED"; tail -5 "$O/abenv_$i.err"; exit 1; }
  python3 - "$v" "$O/abenv_$i.json" <<'PY'
import json, sys
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>24} {b['ms_per_step']:8.3f} ms  latency {b.get('latency_ms')} device {b.get('device_resident_ms')}")
PY
done
