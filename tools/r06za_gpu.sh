# round 6: two trace rounds in flight and the composition columns' all-gathers ahead of the assertion quotient --
# sharded parity first, then the replicated-prefix sweep and the schedule replay at 2^22
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sharded.py \
    tests/test_sharded_multiprocess.py > $O/r06za_sharded_tests.log 2>&1 || { tail -30 $O/r06za_sharded_tests.log; exit 1; }
tail -2 $O/r06za_sharded_tests.log
timeout -k 10 500 python3 tools/shard_model.py --sweep 22 > $O/r06za_split_sweep_2p22.json 2> $O/r06za_split_sweep.err \
    || { tail -20 $O/r06za_split_sweep.err; exit 1; }
grep -v "^\[" $O/r06za_split_sweep.err | tail -40
timeout -k 10 400 python3 tools/shard_model.py --schedule 22 > $O/r06za_shard_schedule_2p22.json 2> $O/r06za_shard_schedule.err \
    || { tail -20 $O/r06za_shard_schedule.err; exit 1; }
tail -9 $O/r06za_shard_schedule.err
