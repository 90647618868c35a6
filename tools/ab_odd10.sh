#!/bin/bash
# 2^21 four-step split: pass-1 lines of 2^11 (base) or 2^10 (variant odd10); parity of the variant, then A/B.
set -eo pipefail
ZKVM_GPU_LIB=encrypt-zkvm_amd/lib/libzkvm_gpu_odd10.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -x -q --timeout 300 --timeout-method thread -k "ntt or x_cipher_2p21" > gpurun_out/odd10_tests.log 2>&1
echo "odd10 parity tests ok"
AB_STEPS=10 BENCH_ARGS="--log-n 21 --inflight 2" bash tools/ab_variants.sh base odd10 base odd10
