#!/bin/bash
# virtual columns: GPU parity + VM suites, then A/B against ZK_VIRTUAL=0
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vm.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_r04s.log 2>&1
rc=$?; tail -3 $O/tests_r04s.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests_r04s.log | head; exit $rc; }
BENCH_ARGS=--ab STEPS=20 bash tools/ab_env.sh - ZK_VIRTUAL=0 - ZK_VIRTUAL=0 - ZK_VIRTUAL=0
