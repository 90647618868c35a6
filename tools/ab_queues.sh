#!/bin/bash
# A/B of the upload-stream layout under HIP's default 4 hardware queues and under 16:
#   own    = a copy stream per prover, compute stream parks on the upload event (round-3 layout)
#   shared = one upload stream per device (P + 1 streams), device-side event wait
#   host   = shared upload stream, the host thread waits for each group's event before enqueueing its kernels
# Each line: ms_per_step (20 proofs), steady_state_ms (100), latency_ms, device_resident_ms, vm_prove_ms.
set -o pipefail
O=gpurun_out
mkdir -p $O
run() {  # name queues stream gate inflight [upload plan]
  GPU_MAX_HW_QUEUES=$2 ZK_UPLOAD_STREAM=$3 ZK_UPLOAD_GATE=$4 ZK_UPLOAD_PLAN=${6:-incr} timeout -k 10 400 python3 bench.py --no-cpu-baseline \
    --no-verify --ab --inflight $5 ${BENCH_ARGS:-} > $O/abq_$1.json 2> $O/abq_$1.err || { echo "$1 FAILED"; tail -5 $O/abq_$1.err; exit 1; }
  python3 - "$1" "$O/abq_$1.json" <<'PY'
import json, sys
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
v = b.get("vm", {})
print(f"{sys.argv[1]:>14} {b['ms_per_step']:7.3f} steady {b.get('steady_state_ms')} lat {b.get('latency_ms')} dev {b.get('device_resident_ms')} "
      f"vm_prove {v.get('vm_prove_ms')} (lat {v.get('vm_prove_latency_ms')}, same {v.get('vm_prove_same_proof')}) pin {b.get('proof_matches_pin')}")
PY
}
for rep in $(seq 1 ${AB_REPS:-2}); do
  run q4_sh_dev_p4 4 shared device 4
  run q4_sh_host_p4 4 shared host 4
  run q4_sh_dev_p3 4 shared device 3
  run q4_sh_host_p3 4 shared host 3
  run q4_sh_dev_p2 4 shared device 2
done
