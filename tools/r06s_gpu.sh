# round 6: the committed tree's clean build on a fresh box -- smoke, the GPU suite, the default bench line
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r06s_smoke.log 2>&1 || { tail -20 $O/r06s_smoke.log; exit 1; }
tail -2 $O/r06s_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r06s_gpu_tests.log 2>&1 || { tail -20 $O/r06s_gpu_tests.log; exit 1; }
tail -2 $O/r06s_gpu_tests.log
timeout -k 10 600 python3 bench.py > $O/r06s_bench.json 2> $O/r06s_bench.err || { tail -20 $O/r06s_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/r06s_bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print(d['ms_per_step'], d['value'], r['frac'], r['compute_frac'], r['traffic_source']['profile_tree_matches'], r['valu_hw']['profile_tree_matches'], d['cpu_baseline']['median_s'], d['mixed_programs']['vs_programs_alone'], d['proof_matches_pin'])"
