#!/bin/bash
# Round-4 session: first-upload-group A/B (latency), then one SQ stall-breakdown pass over one proof.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
STEPS=20 bash tools/ab_env.sh - ZK_UPLOAD_FIRST=1 ZK_UPLOAD_FIRST=2 - ZK_UPLOAD_FIRST=1 ZK_UPLOAD_FIRST=2 > "$O/ab_first.txt" 2>&1 || { cat "$O/ab_first.txt"; exit 1; }
cat "$O/ab_first.txt"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d "$O/pmc_stall" -o st -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --inflight 1 --no-cpu-baseline --no-verify --no-compare > /dev/null 2> "$O/pmc_stall.err" || { tail -5 "$O/pmc_stall.err"; exit 1; }
python3 "$R/tools/pmc_stall.py" "$O/pmc_stall" -o "$O/pmc_stall.md"
find "$O/pmc_stall" -name '*counter_collection.csv' -size +20M -delete || true
