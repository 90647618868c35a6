#!/bin/bash
# evaluator limb sums regrouped: GPU parity/VM suites, then A/B against the previous evaluator (variant "old")
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vm.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_r04y.log 2>&1
rc=$?; tail -3 $O/tests_r04y.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests_r04y.log | head; exit $rc; }
bash tools/ab_variants.sh base old base old base old
