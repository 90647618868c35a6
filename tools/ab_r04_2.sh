#!/bin/bash
# Round-4 A/B session 2: ZK_NTT_GRP=2 at 2^22 (the sizes it changes), then the evaluator's HBM traffic with and
# without the LDS stash (PMC FETCH_SIZE / WRITE_SIZE passes, one proof each, tools/pmc_traffic.py).
set -o pipefail
O=gpurun_out
R=$(pwd)
mkdir -p $O
BENCH_ARGS="--ab --log-n 22 --inflight 2" AB_STEPS=6 bash tools/ab_variants.sh base grp2 base grp2 base grp2 > $O/ab_grp2_2p22.txt 2>&1
cat $O/ab_grp2_2p22.txt
cd /tmp && export TMPDIR=/tmp
for v in base nostash; do
  if [ $v = base ]; then lib=$R/encrypt-zkvm_amd/lib/libzkvm_gpu.so; else lib=$R/encrypt-zkvm_amd/lib/libzkvm_gpu_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    ZKVM_GPU_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$R/$O/pmc_${c}_$v" -o x -- \
      python3 "$R/bench.py" --steps 1 --warmup 0 --inflight 1 --no-cpu-baseline --no-verify --no-compare \
      > /dev/null 2> "$R/$O/pmc_${c}_$v.err" || { echo "pmc $c $v FAILED"; tail -5 "$R/$O/pmc_${c}_$v.err"; exit 1; }
  done
  python3 "$R/tools/pmc_traffic.py" "$R/$O/pmc_FETCH_SIZE_$v" "$R/$O/pmc_WRITE_SIZE_$v" -o "$R/$O/pmc_traffic_$v.json"
  find "$R/$O/pmc_FETCH_SIZE_$v" "$R/$O/pmc_WRITE_SIZE_$v" -name '*counter_collection.csv' -size +20M -delete || true
  python3 - "$R/$O/pmc_traffic_$v.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
pl = d["per_launch_bytes"]
print(sys.argv[2], {k: round(v / 1e9, 3) for k, v in pl.items() if k.startswith(("eval", "ntt", "hash_rows"))})
PY
done
