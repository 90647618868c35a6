set -eo pipefail
mkdir -p gpurun_out
ZKVM_GPU_LIB=encrypt-zkvm_amd/lib/libzkvm_gpu_grp2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "ntt or full_proof or stage_dumps or full_size or 2_22 or 2p23" > gpurun_out/grp2_tests.log 2>&1 || { tail -30 gpurun_out/grp2_tests.log; exit 1; }
tail -1 gpurun_out/grp2_tests.log
ZKVM_GPU_LIB=encrypt-zkvm_amd/lib/libzkvm_gpu_glast.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "ntt or full_proof or stage_dumps" > gpurun_out/glast_tests.log 2>&1 || { tail -30 gpurun_out/glast_tests.log; exit 1; }
tail -1 gpurun_out/glast_tests.log
BENCH_ARGS=--no-compare bash tools/ab_variants.sh base glast grp2 base glast grp2
BENCH_ARGS="--no-compare --log-n 22 --inflight 2" AB_STEPS=6 bash tools/ab_variants.sh base grp2 base grp2
