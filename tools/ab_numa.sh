#!/bin/bash
# A/B of the NUMA binding of the bench's host threads (ZK_NUMA_BIND=0 vs default), alternating on one box.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
for rep in 1 2; do
  for b in 0 1; do
    ZK_NUMA_BIND=$b timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify > "$O/numa_ab_${b}_$rep.json" 2> "$O/numa_ab_${b}_$rep.err"
    python3 -c "import json;d=json.load(open('$O/numa_ab_${b}_$rep.json'));print('bind=$b rep=$rep', d['ms_per_step'], d['device_resident_ms'], d['pageable_host_ms'], d['latency_ms'], d['config']['host_numa_node'])"
  done
done
