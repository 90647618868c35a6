# round 6: sharded tests with the coset-pipelined slices / trace commitment, then the schedule replay at 2^22
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sharded.py tests/test_sharded_multiprocess.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r06w_shard_tests.log 2>&1
rc=$?
tail -5 $O/r06w_shard_tests.log
if [ $rc -ne 0 ]; then echo "sharded tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python3 tools/shard_model.py --schedule 22 > $O/r06w_shard_schedule_2p22.json 2> $O/r06w_shard_schedule.err || { tail -20 $O/r06w_shard_schedule.err; exit 1; }
tail -9 $O/r06w_shard_schedule.err
python3 -c "
import json; d=json.load(open('$O/r06w_shard_schedule_2p22.json'))
for k, v in d['projection'].items(): print(k, json.dumps({g: v[g]['per_rank_ms'] for g in ('2','4','8') if g in v}), json.dumps({g: v[g]['exposed_exchange_ms'] for g in ('2','4','8') if g in v}))"
