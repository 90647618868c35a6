#!/bin/bash
# UNI (wave-uniform twiddle) rounds for 2048-point lines: parity with the variant library, then A/B at 2^21 and 2^23.
set -eo pipefail
ZKVM_GPU_LIB=encrypt-zkvm_amd/lib/libzkvm_gpu_u11.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "ntt or full_size or largest" > gpurun_out/u11_tests.log 2>&1
echo "u11 parity tests ok"
AB_STEPS=10 BENCH_ARGS="--log-n 21 --inflight 2" bash tools/ab_variants.sh base u11 base u11
AB_STEPS=4 BENCH_ARGS="--log-n 23 --inflight 1" bash tools/ab_variants.sh base u11
