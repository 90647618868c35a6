#!/bin/bash
# A/B the prover library variants built by `make variant NAME=...` on the default bench workload:
#   bash tools/ab_variants.sh base name1 name2 ...   ("base" = lib/libzkvm_gpu.so)
# Each variant: one bench line (no CPU baseline, no verification); prints ms_per_step + kernel times.
set -eo pipefail
O=gpurun_out
mkdir -p "$O"
for v in "$@"; do
  if [ "$v" = base ]; then lib=encrypt-zkvm_amd/lib/libzkvm_gpu.so; else lib=encrypt-zkvm_amd/lib/libzkvm_gpu_$v.so; fi
  ZKVM_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify --steps ${AB_STEPS:-20} --warmup ${AB_WARMUP:-12} ${BENCH_ARGS:-} \
    > "$O/ab_$v.json" 2> "$O/ab_$v.err" || { echo "$v FAILED"; tail -5 "$O/ab_$v.err"; exit 1; }
  python3 - "$v" "$O/ab_$v.json" <<'PY'
import json, sys
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = b.get("kernel_ms", {})
print(f"{sys.argv[1]:>12} {b['ms_per_step']:8.3f} ms  latency {b.get('latency_ms')} device {b.get('device_resident_ms')} "
      f"pageable {b.get('pageable_host_ms')}  " + " ".join(f"{n}={v}" for n, v in list(k.items())[:4]))
PY
done
