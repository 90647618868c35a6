#!/bin/bash
# A/B of provers in flight under HIP's default 4 hardware queues and under 16 (one upload stream per device, host-side
# gating; the stream-per-prover, device-side-wait and 7-groups-of-4 layouts this replaced are in
# profiles/r04_ab_queues_pass1.txt and profiles/r04_ab_queues.txt).
# Each line: ms_per_step (20 proofs), steady_state_ms (100), latency_ms, device_resident_ms, vm_prove_ms.
set -o pipefail
O=gpurun_out
mkdir -p $O
run() {  # name queues inflight
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 400 python3 bench.py --no-cpu-baseline \
    --no-verify --ab --inflight $3 ${BENCH_ARGS:-} > $O/abq_$1.json 2> $O/abq_$1.err || { echo "$1 FAILED"; tail -5 $O/abq_$1.err; exit 1; }
  python3 - "$1" "$O/abq_$1.json" <<'PY'
import json, sys
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
v = b.get("vm", {})
print(f"{sys.argv[1]:>14} {b['ms_per_step']:7.3f} steady {b.get('steady_state_ms')} lat {b.get('latency_ms')} dev {b.get('device_resident_ms')} "
      f"vm_prove {v.get('vm_prove_ms')} (lat {v.get('vm_prove_latency_ms')}, same {v.get('vm_prove_same_proof')}) pin {b.get('proof_matches_pin')}")
PY
}
for rep in $(seq 1 ${AB_REPS:-2}); do
  run q4_p2 4 2
  run q4_p3 4 3
  run q4_p4 4 4
  run q16_p3 16 3
  run q16_p4 16 4
done
