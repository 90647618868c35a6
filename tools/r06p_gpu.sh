# round 6: openings storage reused on the sharded path -- sharded tests, the lead window at G = 8, schedule replay
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sharded.py tests/test_sharded_multiprocess.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r06p_shard_tests.log 2>&1
rc=$?
tail -3 $O/r06p_shard_tests.log
if [ $rc -ne 0 ]; then echo "sharded tests rc=$rc: stopping"; exit $rc; fi
bash tools/r06o_gpu.sh && cp $O/r06o_lead_window_g8.txt $O/r06p_lead_window_g8.txt || exit 1
timeout -k 10 400 python3 tools/shard_model.py --schedule 22 > $O/r06p_shard_schedule_2p22.json 2> $O/r06p_shard_schedule.err || { tail -20 $O/r06p_shard_schedule.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r06p_shard_schedule_2p22.json'))
for k, v in d['projection'].items(): print(k, json.dumps({g: (v[g]['per_rank_ms'], v[g]['lead_only_ms']) for g in ('2','4','8') if g in v}))"
