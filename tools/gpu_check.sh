#!/bin/bash
# One GPU-box check: the full -m gpu parity suite, then the default bench line (and any extra bench
# arguments given).  Usage (via gpurun, from the repo root):  bash tools/gpu_check.sh <tag> [bench args]
set -eo pipefail
TAG=${1:-check}
shift || true
O=gpurun_out
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests_$TAG.log" 2>&1 \
  || { tail -40 "$O/gpu_tests_$TAG.log"; exit 1; }
tail -1 "$O/gpu_tests_$TAG.log"
timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err" \
  || { tail -20 "$O/bench_$TAG.err"; exit 1; }
python3 - "$O/bench_$TAG.json" <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("ms_per_step", b["ms_per_step"], "value", b["value"])
print("kernel_ms", b.get("kernel_ms"))
print("stage_ms", b.get("stage_ms"))
PY
