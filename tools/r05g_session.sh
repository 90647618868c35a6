#!/bin/bash
# Round-5 session g (final tree, after tools/gpu_profile.sh r05f tests nobench): the default bench line, config 5, the
# one-call latency timeline, and configs[3]'s 2^22 proof on one GPU.
set -eo pipefail
R=$(pwd)
O=$R/gpurun_out
mkdir -p "$O"
timeout -k 10 600 python3 bench.py > "$O/bench_r05g.json" 2> "$O/bench_r05g.err" || { tail -20 "$O/bench_r05g.err"; exit 1; }
echo "bench ok"
timeout -k 10 400 python3 bench.py --config5 --no-cpu-baseline > "$O/bench_c5_r05g.json" 2> "$O/bench_c5_r05g.err" \
  || { tail -20 "$O/bench_c5_r05g.err"; exit 1; }
echo "config5 ok"
timeout -k 10 400 python3 bench.py --log-n 22 --steps 6 --inflight 1 --no-cpu-baseline --no-compare --sharded-log-n 0 \
  > "$O/bench_2p22_r05g.json" 2> "$O/bench_2p22_r05g.err" || { tail -20 "$O/bench_2p22_r05g.err"; exit 1; }
echo "2^22 ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/lat_r05g" -o lat -- \
  python3 "$R/tools/latency_timeline.py" --out "$O/lat_marks_r05g.json" > "$O/lat_run_r05g.log" 2>&1
python3 "$R/tools/latency_timeline.py" --analyze "$O/lat_r05g" --marks "$O/lat_marks_r05g.json" > "$O/lat_timeline_r05g.json"
find "$O/lat_r05g" -name '*.csv' -size +30M -delete || true
cat "$O/bench_r05g.json"
