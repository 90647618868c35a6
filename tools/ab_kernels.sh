#!/bin/bash
# Kernel-variant A/B (libraries from `make variant`): the variants' NTT / evaluator / full-proof / pin tests, then
# alternating bench lines (--ab: steady state, device-resident, latency) at 2^20, and grp2 at 2^22.
set -o pipefail
O=gpurun_out
mkdir -p $O
for v in glast nostash grp2; do
  sel="ntt or full_proof or stage_dumps or plug or sparse or config1 or full_size"
  [ $v = grp2 ] && sel="ntt or full_size or 2p23"
  ZKVM_GPU_LIB=encrypt-zkvm_amd/lib/libzkvm_gpu_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "$sel" > $O/abk_tests_$v.log 2>&1 || { echo "$v tests FAILED"; tail -30 $O/abk_tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 $O/abk_tests_$v.log)"
done
BENCH_ARGS="--ab" bash tools/ab_variants.sh base glast nostash base glast nostash
BENCH_ARGS="--ab --log-n 22 --inflight 2" AB_STEPS=6 bash tools/ab_variants.sh base grp2 base grp2
