#!/bin/bash
# One GPU-box session (kernel traces and counters with one prover, so no launch overlaps another): parity tests, rocprofv3 kernel-trace stats of the bench, two PMC passes
# (FETCH_SIZE / WRITE_SIZE, separately) -> pmc_traffic.json, then the default bench line.
# Usage (from the repo root, via gpurun):  bash tools/gpu_profile.sh <tag> [tests|notests] [bench|nobench]
# (nobench: the profiles and counters only; the bench lines in a session of their own)
set -eo pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
BENCH_ARGS="--steps 4 --warmup 2 --inflight 1 --no-cpu-baseline --no-verify --no-compare --upload-schedule throughput"

if [ "${2:-tests}" = "tests" ]; then
  (cd "$R" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$O/gpu_tests_$TAG.log" 2>&1)
  echo "gpu tests ok"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o "$TAG" -- \
  python3 "$R/bench.py" $BENCH_ARGS > "$O/prof_bench_$TAG.json" 2> "$O/prof_bench_$TAG.err"
echo "kernel trace ok"
# (3 warm-up proofs first: the profiled last proof is a steady-state one, column hints in use; pmc_traffic.py counts
# that proof's dispatches only, against its algorithmic bytes from the same run's bench line.  One prover, on the
# throughput upload schedule: the launches of the default line's three-in-flight proofs, not of one proof alone)
PMC_ARGS="--steps 1 --warmup 3 --inflight 1 --no-cpu-baseline --no-verify --no-compare --input-sets 1 --upload-schedule throughput"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch_$TAG" -o f -- \
  python3 "$R/bench.py" $PMC_ARGS > "$O/pmc_fetch_bench_$TAG.json" 2> "$O/pmc_fetch_$TAG.err"
echo "pmc fetch ok"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write_$TAG" -o w -- \
  python3 "$R/bench.py" $PMC_ARGS > /dev/null 2> "$O/pmc_write_$TAG.err"
echo "pmc write ok"
python3 "$R/tools/pmc_traffic.py" "$O/pmc_fetch_$TAG" "$O/pmc_write_$TAG" --bench "$O/pmc_fetch_bench_$TAG.json" \
  -o "$O/pmc_traffic_$TAG.json"
cp "$O/pmc_traffic_$TAG.json" "$R/profiles/pmc_traffic.json"
# VALU issue rate: 6 SQ + 2 GRBM counters, one pass of its own
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_LDS SQ_BUSY_CYCLES \
  SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$O/pmc_sq_$TAG" -o sq -- \
  python3 "$R/bench.py" $PMC_ARGS > /dev/null 2> "$O/pmc_sq_$TAG.err"
python3 "$R/tools/pmc_valu.py" "$O/pmc_sq_$TAG" -o "$O/pmc_valu_$TAG.md" -j "$O/pmc_valu_$TAG.json"
cp "$O/pmc_valu_$TAG.json" "$R/profiles/pmc_valu.json"
echo "pmc sq ok"
# where the waves spend their cycles (8 SQ counters, one pass): waitcnt / barrier, issue stall, issuing
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d "$O/pmc_stall_$TAG" -o st -- \
  python3 "$R/bench.py" $PMC_ARGS > /dev/null 2> "$O/pmc_stall_$TAG.err"
python3 "$R/tools/pmc_stall.py" "$O/pmc_stall_$TAG" -o "$O/pmc_stall_$TAG.md"
echo "pmc stall ok"
# keep only the summaries (the per-dispatch counter CSVs are large)
find "$O/pmc_fetch_$TAG" "$O/pmc_write_$TAG" -name '*counter_collection.csv' -size +20M -delete || true
BENCH=${3:-bench}
if [ "$BENCH" = bench ]; then
  (cd "$R" && timeout -k 10 600 python3 bench.py > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err")
  echo "bench ok"
fi
# config 5 (128-bit options, quadratic extension): kernel trace + bench line
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c5_$TAG" -o "c5_$TAG" -- \
  python3 "$R/bench.py" --config5 $BENCH_ARGS > "$O/prof_bench_c5_$TAG.json" 2> "$O/prof_bench_c5_$TAG.err"
echo "config5 kernel trace ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch_c5_$TAG" -o f -- \
  python3 "$R/bench.py" --config5 $PMC_ARGS > "$O/pmc_fetch_bench_c5_$TAG.json" 2> "$O/pmc_fetch_c5_$TAG.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write_c5_$TAG" -o w -- \
  python3 "$R/bench.py" --config5 $PMC_ARGS > /dev/null 2> "$O/pmc_write_c5_$TAG.err"
python3 "$R/tools/pmc_traffic.py" "$O/pmc_fetch_c5_$TAG" "$O/pmc_write_c5_$TAG" --bench "$O/pmc_fetch_bench_c5_$TAG.json" \
  -o "$O/pmc_traffic_c5_$TAG.json"
cp "$O/pmc_traffic_c5_$TAG.json" "$R/profiles/pmc_traffic_config5.json"
find "$O/pmc_fetch_c5_$TAG" "$O/pmc_write_c5_$TAG" -name '*counter_collection.csv' -size +20M -delete || true
echo "config5 pmc ok"
if [ "$BENCH" = bench ]; then
  (cd "$R" && timeout -k 10 600 python3 bench.py --config5 --no-cpu-baseline > "$O/bench_c5_$TAG.json" 2> "$O/bench_c5_$TAG.err")
  echo "config5 bench ok"
  cat "$O/bench_$TAG.json"
fi
