#!/bin/bash
# Round-5 session d: single-call latency A/B of the upload order (31 calls per process, variants alternating, 3
# rounds), then the multi-GPU bench flow rehearsed at N = 4 on the one GPU (torchrun, TCP host group, host-exchange
# sharded leg).
set -eo pipefail
O=gpurun_out
mkdir -p "$O"
for rep in 1 2 3; do
  for v in "base:" "f1:ZK_UPLOAD_FIRST=1" "f2:ZK_UPLOAD_FIRST=2" "nf:ZK_NARROW_FIRST=1"; do
    name=${v%%:*}; envs=${v#*:}
    echo -n "$name $rep " && env $envs timeout -k 10 200 python3 tools/latency_ab.py 31 2>> "$O/latab.err"
  done
done | tee "$O/latency_ab.txt"
bash tools/rehearse_multi.sh 4
