#!/bin/bash
# clock derivation: GPU parity + VM suites, then the bench line
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vm.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_r04k.log 2>&1
rc=$?; tail -3 $O/tests_r04k.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests_r04k.log | head; exit $rc; }
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench_r04k.json 2> $O/bench_r04k.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_r04k.json'));print(d['ms_per_step'],d['latency_ms'],d['device_resident_ms'],d['steady_state_ms'],d['proof_matches_pin'],d['trace_upload'],d['kernel_ms'])"
