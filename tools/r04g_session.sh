set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --steps 8 --no-cpu-baseline > gpurun_out/bench_r04g.json 2> gpurun_out/bench_r04g.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/bench_r04g.json'));print(d['ms_per_step'],d['proof_matches_pin'],d['roofline'])"
bash tools/shard_check.sh r04g || exit 1
bash tools/rehearse_multi.sh 2
