#!/bin/bash
# Device VM trace generator + vm::prove on the GPU box: its tests, then one bench line (no CPU baseline).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_vm.py "tests/test_gpu_parity.py::test_host_trace_memory_outlives_its_owner" \
  -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/vm_tests.log 2>&1
rc=$?
tail -25 gpurun_out/vm_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/vm_bench.json 2> gpurun_out/vm_bench.err
rc=$?
tail -3 gpurun_out/vm_bench.err
exit $rc
