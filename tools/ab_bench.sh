# A/B timing of library variants on the GPU box: bash tools/ab_bench.sh [variant ...]
# A variant is <lib>[%VAR=value[%VAR=value...]]: <lib> "new" is the in-tree
# corda_amd/libcordagpu.so, any other name abvar/libcg_<lib>.so; the VAR=value pairs
# are set in the bench's environment (e.g. new%CORDA_AMD_ED_SPLIT=1).  Bench arguments
# come from $AB_ARGS.  Each variant runs twice, interleaved; results go to gpurun_out/ab.txt.
set -e
names=${*:-base new}
for rep in $(seq 1 ${AB_REPS:-2}); do
  for v in $names; do
    lib=${v%%\%*}
    envs=()
    if [[ $v == *%* ]]; then IFS=% read -r -a envs <<< "${v#*%}"; fi
    if [ "$lib" = new ]; then unset CORDA_AMD_LIB; else export CORDA_AMD_LIB=$PWD/abvar/libcg_$lib.so; fi
    tag=${v//[%=]/_}
    env "${envs[@]}" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra --latency-runs 1 \
      $AB_ARGS > gpurun_out/ab_$tag.log 2>&1
    python -c "import json; d=json.loads(open('gpurun_out/ab_$tag.log').read().splitlines()[-1]); print('$v', d['value'], {k:v['avg_launch_ms'] for k,v in d['kernels'].items()})" >> gpurun_out/ab.txt
  done
done
