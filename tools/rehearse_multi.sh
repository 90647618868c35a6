#!/bin/bash
# Rehearse the driver's multi-GPU bench flow (torchrun, N ranks) on a one-GPU box: ZK_BENCH_REHEARSE=1 puts every
# rank on the one GPU and the sharded leg on the host-exchange communicator over the TCP host group (no torch).
# Usage (GPU box): bash tools/rehearse_multi.sh N
set -eo pipefail
N=${1:-2}
O=gpurun_out
mkdir -p "$O"
ZK_BENCH_REHEARSE=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus "$N" --steps 8 --warmup 2 \
  > "$O/rehearse_$N.json" 2> "$O/rehearse_$N.err"
python3 - "$O/rehearse_$N.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sh = d.get("sharded", {})
print("n_gpus", d["n_gpus"], "value", d["value"], "ms_per_step", d["ms_per_step"], "verified", d.get("proof_verified_by_oracle"))
print("replica pin", d.get("proof_matches_pin"), "all ranks verified", d.get("all_ranks_verified_by_zk_verify"))
print("sharded", {k: sh.get(k) for k in ("n_ranks", "ms_per_proof", "device_resident_ms_per_proof", "vm_prove_ms_per_proof",
                                         "device_resident_and_vm_prove_same_proof", "proof_matches_pin",
                                         "all_ranks_verified_by_zk_verify", "error")})
print("exchange", {k: v for k, v in (sh.get("exchange") or {}).items()})
PY
