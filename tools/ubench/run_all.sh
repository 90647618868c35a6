#!/bin/bash
# Run every microbenchmark / lab in this directory on one GPU box (from the repo root):
#   bash tools/ubench/run_all.sh  ->  gpurun_out/ubench_<name>.txt
set -eo pipefail
O=gpurun_out
mkdir -p "$O"
for b in instr_ubench instr2_ubench instr3_ubench fmul_ilp fmul_lab fadd_lab b3_lab ntt_lab; do
  timeout -k 5 90 ./tools/ubench/$b > "$O/ubench_$b.txt" 2>&1 || { echo "$b failed"; tail -5 "$O/ubench_$b.txt"; exit 1; }
  echo "== $b"; cat "$O/ubench_$b.txt"
done
