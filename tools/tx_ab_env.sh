# Tx pipeline A/B of one environment switch: bash tools/tx_ab_env.sh VAR "v1 v2"  -> gpurun_out/txe/summary.txt
set -e
mkdir -p gpurun_out/txe
for rep in 1 2; do
  for v in $2; do
    env $1=$v timeout -k 10 200 python -u bench.py --workload tx --steps 5 --warmup 1 --no-cpu-baseline --latency-runs 1 > gpurun_out/txe/${v}_$rep.log 2>&1
    python -c "import json; d=json.loads(open('gpurun_out/txe/${v}_$rep.log').read().splitlines()[-1]); print('$1=$v', d['value'], d['ms_per_step'])" >> gpurun_out/txe/summary.txt
  done
done
