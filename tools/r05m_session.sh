#!/bin/bash
# Round-5 session m: one zk_vm_prove call as a timeline (kernel + copy trace), and the vm latency A/B of the stack pass
# with a compile-time ciphertext width (new build) -- numbers only, the pass is host code.
set -eo pipefail
R=$(pwd)
O=$R/gpurun_out
mkdir -p "$O"
timeout -k 10 300 python3 tools/vm_latency_ab.py 31 > "$O/r05m_vm_latency.txt"
cat "$O/r05m_vm_latency.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/lat_vm_r05m" -o lat -- \
  python3 "$R/tools/latency_timeline.py" --vm --out "$O/lat_vm_marks_r05m.json" > "$O/lat_vm_run_r05m.log" 2>&1
python3 "$R/tools/latency_timeline.py" --analyze "$O/lat_vm_r05m" --marks "$O/lat_vm_marks_r05m.json" > "$O/lat_vm_timeline_r05m.json"
find "$O/lat_vm_r05m" -name '*.csv' -size +30M -delete || true
cat "$O/lat_vm_timeline_r05m.json" | head -30
