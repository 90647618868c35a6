# round 6: the replicated-prefix sweep again with block coset ownership
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python3 tools/shard_model.py --sweep 22 > $O/r06v_split_sweep_2p22.json 2> $O/r06v_split_sweep.err
rc=$?
cat $O/r06v_split_sweep.err | grep -v "^\[" | tail -50
exit $rc
