# round 6: GPU suite on the current tree, the sharded schedule model at 2^22, then A/B of the carry-chain asm
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/r06c_gpu_tests.log 2>&1
rc=$?
tail -5 $O/r06c_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python3 tools/shard_model.py --schedule 22 > $O/r06c_shard_schedule_2p22.json 2> $O/r06c_shard_schedule.err || { tail -20 $O/r06c_shard_schedule.err; exit 1; }
tail -9 $O/r06c_shard_schedule.err
python3 -c "
import json; d=json.load(open('$O/r06c_shard_schedule_2p22.json'))
for k, v in d['projection'].items(): print(k, json.dumps(v))"
AB_STEPS=60 bash tools/ab_variants.sh base nofold2 noasm base nofold2 noasm base nofold2 noasm > $O/r06c_ab.txt 2>&1
cat $O/r06c_ab.txt
