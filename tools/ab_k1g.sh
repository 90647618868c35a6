set -eo pipefail
ZKVM_GPU_LIB=encrypt-zkvm_amd/lib/libzkvm_gpu_k1g.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "ntt or full_size" > gpurun_out/k1g_tests.log 2>&1
echo "tests ok"
AB_STEPS=20 bash tools/ab_variants.sh base k1g base k1g
AB_STEPS=6 BENCH_ARGS="--log-n 22 --inflight 2" bash tools/ab_variants.sh base k1g base k1g
