# round 6 final evidence on the final tree: the sharded schedule replay at 2^22 first (bench.py's model record reads
# it from profiles/), then tools/final_profile.sh (GPU suite, kernel traces, PMC traffic / VALU / stall passes, bench
# lines at configs[2] / configs[4] / 2^22, one-call timelines) and the driver's multi-rank bench flow rehearsed with 2
# ranks on the one GPU
set -eo pipefail
TAG=${1:-r06z}
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python3 tools/shard_model.py --schedule 22 > $O/${TAG}_shard_schedule_2p22.json 2> $O/${TAG}_shard_schedule.err || { tail -20 $O/${TAG}_shard_schedule.err; exit 1; }
tail -9 $O/${TAG}_shard_schedule.err
cp $O/${TAG}_shard_schedule_2p22.json profiles/${TAG}_shard_schedule_2p22.json
bash tools/final_profile.sh $TAG
bash tools/rehearse_multi.sh 2
