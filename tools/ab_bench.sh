set -e
for v in base new base new; do
  if [ $v = base ]; then export CORDA_AMD_LIB=$PWD/variants/libcg_base.so; else unset CORDA_AMD_LIB; fi
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-runs 1 > gpurun_out/ab_$v.log 2>&1
  python -c "import json; d=json.loads(open('gpurun_out/ab_$v.log').read().splitlines()[-1]); print('$v', d['value'], {k:v['avg_launch_ms'] for k,v in d['kernels'].items()})" >> gpurun_out/ab.txt
done
