# Tx pipeline chunk-count sweep on the GPU box: bash tools/tx_chunks.sh [counts...]
# -> gpurun_out/txc/summary.txt (one "chunks tx/s ms/step" line per count)
set -e
mkdir -p gpurun_out/txc
for c in ${*:-4 5 6}; do
  CORDA_AMD_TX_CHUNKS=$c timeout -k 10 200 python -u bench.py --workload tx --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/txc/c$c.log 2>&1
  python -c "import json; d=json.loads(open('gpurun_out/txc/c$c.log').read().splitlines()[-1]); print($c, d['value'], d['ms_per_step'])" >> gpurun_out/txc/summary.txt
done
