#!/bin/bash
# one single-threaded oracle proof of configs[2]'s 2^20 trace on the GPU box's host (no GPU used), with a heartbeat
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python3 tools/cpu_baseline_2p20.py 1 > $O/cpu_2p20.json 2> $O/cpu_2p20.err &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; date +%s >> $O/cpu_2p20.ticks; echo "running $(($(date +%s) % 100000))"; done
wait $pid
rc=$?
cat $O/cpu_2p20.json
exit $rc
