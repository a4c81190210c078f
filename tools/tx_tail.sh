# Tx pipeline: last-chunk size sweep (CORDA_AMD_TX_TAIL = fraction of a regular chunk)
#   bash tools/tx_tail.sh "6:1.0 6:0.5 7:0.5"  -> gpurun_out/txt/summary.txt
set -e
mkdir -p gpurun_out/txt
for kv in ${1:-6:1.0 6:0.6 6:0.4}; do
  k=${kv%%:*}; t=${kv##*:}
  for rep in 1 2; do
    CORDA_AMD_TX_CHUNKS=$k CORDA_AMD_TX_TAIL=$t timeout -k 10 200 python -u bench.py --workload tx --steps 5 --warmup 1 --no-cpu-baseline --latency-runs 1 > gpurun_out/txt/c${k}_t${t}_$rep.log 2>&1
    python -c "import json; d=json.loads(open('gpurun_out/txt/c${k}_t${t}_$rep.log').read().splitlines()[-1]); print('$k', '$t', d['value'], d['ms_per_step'])" >> gpurun_out/txt/summary.txt
  done
done
