#!/bin/bash
# Round-5 session j: the latency upload schedule (a proof alone on its device) against the throughput one
# (ZK_LATENCY_SCHED=0): one-call latency A/B (3 x 31 calls), the GPU suite, bench A/B, a one-call timeline.
set -eo pipefail
O=gpurun_out
mkdir -p "$O"
: > "$O/r05j_latency_ab.txt"
for k in 1 2 3; do
  for v in "thr:ZK_LATENCY_SCHED=0" "lat:"; do
    name=${v%%:*}; envs=${v#*:}
    echo -n "$name $k " >> "$O/r05j_latency_ab.txt"
    timeout -k 10 120 env $envs python3 tools/latency_ab.py 31 >> "$O/r05j_latency_ab.txt"
  done
done
cat "$O/r05j_latency_ab.txt"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 \
  --timeout-method thread > "$O/gpu_tests_r05j.log" 2>&1 || { tail -60 "$O/gpu_tests_r05j.log"; exit 1; }
tail -1 "$O/gpu_tests_r05j.log"
AB="--no-cpu-baseline --ab --no-verify --sharded-log-n 0 --steps 30"
: > "$O/r05j_bench_ab.txt"
for k in 1 2; do
  for v in "thr:ZK_LATENCY_SCHED=0" "lat:"; do
    name=${v%%:*}; envs=${v#*:}
    timeout -k 10 300 env $envs python3 bench.py $AB > "$O/r05j_ab_${name}_$k.json" 2>> "$O/r05j_ab.err"
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d.get('latency_ms'), d.get('device_resident_ms'), d.get('steady_state_ms'))" \
      "$O/r05j_ab_${name}_$k.json" "$name $k" >> "$O/r05j_bench_ab.txt"
  done
done
cat "$O/r05j_bench_ab.txt"
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d "$R/$O/lat_r05j" -o lat -- python3 "$R/tools/latency_timeline.py" --out "$R/$O/lat_marks_r05j.json" > "$R/$O/lat_run_r05j.log" 2>&1
python3 "$R/tools/latency_timeline.py" --analyze "$R/$O/lat_r05j" --marks "$R/$O/lat_marks_r05j.json" > "$R/$O/lat_timeline_r05j.json"
find "$R/$O/lat_r05j" -name '*.csv' -size +30M -delete || true
