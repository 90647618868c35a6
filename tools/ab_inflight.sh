set -eo pipefail
for i in 1 2; do
  for P in 3 4; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify --steps 24 --warmup 6 --inflight $P > gpurun_out/abif_$P.json 2> gpurun_out/abif_$P.err
    python3 -c "import json,sys; b=json.loads(open('gpurun_out/abif_$P.json').read().strip().splitlines()[-1]); print('inflight $P', b['ms_per_step'], 'latency', b['latency_ms'], 'device', b['device_resident_ms'], 'pageable', b['pageable_host_ms'])"
  done
done
