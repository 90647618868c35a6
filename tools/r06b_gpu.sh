# round 6: paired final reductions (ws_fold2) -- parity, then A/B against the add/sub asm alone and the compiler's
# chains; the sharded schedule model at 2^22 (measurement-mode loopback, tools/shard_model.py --schedule)
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/r06b_parity.log 2>&1 || { tail -30 $O/r06b_parity.log; exit 1; }
tail -1 $O/r06b_parity.log
AB_STEPS=60 bash tools/ab_variants.sh base nofold2 noasm base nofold2 noasm base nofold2 noasm > $O/r06b_ab_fold2.txt 2>&1
cat $O/r06b_ab_fold2.txt
timeout -k 10 400 python3 tools/shard_model.py --schedule 22 > $O/r06b_shard_schedule_2p22.json 2> $O/r06b_shard_schedule.err || { tail -20 $O/r06b_shard_schedule.err; exit 1; }
tail -12 $O/r06b_shard_schedule.err
python3 -c "
import json; d=json.load(open('$O/r06b_shard_schedule_2p22.json'))
for k, v in d['projection'].items(): print(k, json.dumps(v))"
