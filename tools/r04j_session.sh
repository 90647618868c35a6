#!/bin/bash
# sparse-fill kernel: the hint / pin tests, then A/B-free bench line
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vm.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sparse or narrow or pin or full_size or large or smoke or golden" > $O/tests_r04j.log 2>&1
rc=$?; tail -3 $O/tests_r04j.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench_r04j.json 2> $O/bench_r04j.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_r04j.json'));print(d['ms_per_step'],d['latency_ms'],d['device_resident_ms'],d['proof_matches_pin'],d['kernel_ms'],d['roofline']['frac'],d['vm']['vm_prove_ms'])"
