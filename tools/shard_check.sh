#!/bin/bash
# Sharded-prover check on one GPU box: the loopback and multi-process sharded tests, then the measured loopback
# decomposition at 2^22 (tools/shard_model.py).  Usage (repo root, via gpurun): bash tools/shard_check.sh <tag>
set -eo pipefail
TAG=${1:-shard}
O=gpurun_out
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_sharded.py tests/test_sharded_multiprocess.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$O/shard_tests_$TAG.log" 2>&1 || { tail -40 "$O/shard_tests_$TAG.log"; exit 1; }
tail -1 "$O/shard_tests_$TAG.log"
timeout -k 10 400 python3 tools/shard_model.py 22 3 > "$O/shard_model_$TAG.json" 2> "$O/shard_model_$TAG.err" \
  || { tail -20 "$O/shard_model_$TAG.err"; exit 1; }
cat "$O/shard_model_$TAG.err"
python3 -c "import json; d=json.load(open('$O/shard_model_$TAG.json')); print('fit', d['fit'], 'fit_host', d['fit_host'])"
