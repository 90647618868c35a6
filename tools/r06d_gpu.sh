# round 6: the trace-split sweep of the sharded schedule model at 2^22 (measurement-mode loopback), sharded tests
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python3 tools/shard_model.py --sweep 22 > $O/r06d_split_sweep_2p22.json 2> $O/r06d_split_sweep.err || { tail -20 $O/r06d_split_sweep.err; exit 1; }
cat $O/r06d_split_sweep.err
timeout -k 10 500 python -u -m pytest tests/test_sharded.py tests/test_sharded_multiprocess.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/r06d_shard_tests.log 2>&1
tail -3 $O/r06d_shard_tests.log
