#!/bin/bash
# Round-5 GPU session: the -m gpu suite, smoke, the default bench line, the runtime A/B (the library's own /opt/rocm
# HIP runtime + RCCL against torch's bundled copies, two pairs), the multi-GPU rehearsal at N = 2.
# Usage (via gpurun, from the repo root):  bash tools/r05_check.sh <tag> [tests|notests]
set -eo pipefail
TAG=${1:-r05}
O=gpurun_out
mkdir -p "$O"
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread \
    > "$O/gpu_tests_$TAG.log" 2>&1 || { tail -60 "$O/gpu_tests_$TAG.log"; exit 1; }
  tail -1 "$O/gpu_tests_$TAG.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$TAG.log" 2>&1 \
    || { tail -30 "$O/smoke_$TAG.log"; exit 1; }
  tail -1 "$O/smoke_$TAG.log"
fi
timeout -k 10 600 python3 bench.py > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err" || { tail -30 "$O/bench_$TAG.err"; exit 1; }
echo "bench ok"
AB="--no-cpu-baseline --no-compare --no-verify --sharded-log-n 0 --steps 20"
for k in 1 2; do
  timeout -k 10 300 python3 bench.py $AB > "$O/ab_rt_linked_${TAG}_$k.json" 2>> "$O/ab_rt_$TAG.err"
  timeout -k 10 300 python3 bench.py $AB --torch-runtime > "$O/ab_rt_torch_${TAG}_$k.json" 2>> "$O/ab_rt_$TAG.err"
  echo "runtime A/B pair $k ok"
done
python3 - "$O" "$TAG" <<'PY'
import json, sys
O, tag = sys.argv[1:]
for k in (1, 2):
    for v in ("linked", "torch"):
        d = json.loads(open(f"{O}/ab_rt_{v}_{tag}_{k}.json").read().strip().splitlines()[-1])
        print(v, k, d["ms_per_step"], d["runtime"]["hip_runtime"], d["runtime"]["hip_runtime_version"],
              d["runtime"]["rccl_version"], d.get("proof_matches_pin"))
PY
bash tools/rehearse_multi.sh 2
cat "$O/bench_$TAG.json"
