#!/bin/bash
# Round-5 session b: the wave-local NTT rounds (ZK_NTT_WL, default build) -- the GPU suite, an A/B against the
# barrier-per-round build (lib/libzkvm_gpu_nowl.so), and the one-call latency timeline.
set -eo pipefail
TAG=${1:-r05b}
R=$(pwd)
O=$R/gpurun_out
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread \
  > "$O/gpu_tests_$TAG.log" 2>&1 || { tail -60 "$O/gpu_tests_$TAG.log"; exit 1; }
tail -1 "$O/gpu_tests_$TAG.log"
BENCH_ARGS="--ab --sharded-log-n 0" bash tools/ab_variants.sh base nowl base nowl base nowl | tee "$O/ab_wl_$TAG.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/lat_$TAG" -o lat -- \
  python3 "$R/tools/latency_timeline.py" --out "$O/lat_marks_$TAG.json" > "$O/lat_run_$TAG.log" 2>&1 \
  || { tail -20 "$O/lat_run_$TAG.log"; exit 1; }
python3 "$R/tools/latency_timeline.py" --analyze "$O/lat_$TAG" --marks "$O/lat_marks_$TAG.json" > "$O/lat_timeline_$TAG.json"
cat "$O/lat_timeline_$TAG.json"
find "$O/lat_$TAG" -name '*.csv' -size +30M -delete || true
