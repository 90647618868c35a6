# round 6: in-place trace rounds issued ahead of the previous round's extension -- sharded parity, schedule replay
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sharded.py \
    tests/test_sharded_multiprocess.py > $O/r06zb_sharded_tests.log 2>&1 || { tail -30 $O/r06zb_sharded_tests.log; exit 1; }
tail -2 $O/r06zb_sharded_tests.log
timeout -k 10 400 python3 tools/shard_model.py --schedule 22 > $O/r06zb_shard_schedule_2p22.json 2> $O/r06zb_shard_schedule.err \
    || { tail -20 $O/r06zb_shard_schedule.err; exit 1; }
tail -9 $O/r06zb_shard_schedule.err
