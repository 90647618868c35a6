# round 6: the replicated-prefix sweep on the final schedule (two trace rounds in flight, rounds issued ahead)
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python3 tools/shard_model.py --sweep 22 > $O/r06zc_split_sweep_2p22.json 2> $O/r06zc_split_sweep.err \
    || { tail -20 $O/r06zc_split_sweep.err; exit 1; }
grep -v "^\[" $O/r06zc_split_sweep.err | tail -40
