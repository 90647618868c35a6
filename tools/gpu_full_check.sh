#!/bin/bash
# The whole -m gpu suite (one test per line in the log as it completes), then the default bench line.
# Usage (via gpurun):  bash tools/gpu_full_check.sh <tag> [bench args]
set -o pipefail
TAG=${1:-check}
shift || true
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/gpu_tests_$TAG.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/gpu_tests_$TAG.log | head -20; exit $rc; }
timeout -k 10 400 python3 bench.py --no-cpu-baseline "$@" > $O/bench_$TAG.json 2> $O/bench_$TAG.err
rc=$?
tail -2 $O/bench_$TAG.err
exit $rc
