# round 6 evidence: tools/final_profile.sh (GPU suite, kernel traces, PMC passes, bench lines, 2^22, timelines),
# then the sharded schedule model at 2^22 with the per-world trace split defaults
set -eo pipefail
bash tools/final_profile.sh r06
O=gpurun_out
timeout -k 10 400 python3 tools/shard_model.py --schedule 22 > $O/r06e_shard_schedule_2p22.json 2> $O/r06e_shard_schedule.err || { tail -20 $O/r06e_shard_schedule.err; exit 1; }
tail -9 $O/r06e_shard_schedule.err
