#!/bin/bash
# The end-of-round evidence on one box: tools/gpu_profile.sh (GPU suite, kernel traces, PMC traffic / VALU / stall
# passes, bench lines at configs[2] and configs[4]), then configs[3]'s 2^22 proof on one GPU and the one-call
# timelines of prove() and vm::prove.  Usage (via gpurun, repo root): bash tools/final_profile.sh <tag>
set -eo pipefail
TAG=${1:-final}
R=$(pwd)
O=$R/gpurun_out
bash tools/gpu_profile.sh "$TAG" tests bench
timeout -k 10 400 python3 bench.py --log-n 22 --steps 6 --inflight 1 --no-cpu-baseline --no-compare --sharded-log-n 0 \
  > "$O/bench_2p22_$TAG.json" 2> "$O/bench_2p22_$TAG.err" || { tail -20 "$O/bench_2p22_$TAG.err"; exit 1; }
echo "2^22 ok"
cd /tmp && export TMPDIR=/tmp
for m in host vm; do
  flag=""; [ $m = vm ] && flag="--vm"
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/lat_${m}_$TAG" -o lat -- \
    python3 "$R/tools/latency_timeline.py" $flag --out "$O/lat_${m}_marks_$TAG.json" > "$O/lat_${m}_run_$TAG.log" 2>&1
  python3 "$R/tools/latency_timeline.py" --analyze "$O/lat_${m}_$TAG" --marks "$O/lat_${m}_marks_$TAG.json" \
    > "$O/lat_${m}_timeline_$TAG.json"
  find "$O/lat_${m}_$TAG" -name '*.csv' -size +30M -delete || true
done
echo "timelines ok"
