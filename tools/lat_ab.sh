#!/bin/bash
# Host-buffer latency A/B of library variants on the GPU box (tools/e2e_sweep.py, library
# defaults, pageable inputs): bash tools/lat_ab.sh <tag> [variant ...] with variants as in
# tools/ab_bench.sh (<lib>[%VAR=value...]); sizes from $LAT_SIZES, $AB_REPS interleaved
# repetitions; results gpurun_out/<tag>/sweep_<variant>_<rep>.json.
set -e
tag=${1:?tag}; shift
sizes=${LAT_SIZES:-4096,8192,16384,32768}
mkdir -p gpurun_out/$tag
for rep in $(seq 1 ${AB_REPS:-2}); do
  for v in "$@"; do
    lib=${v%%\%*}
    envs=()
    if [[ $v == *%* ]]; then IFS=% read -r -a envs <<< "${v#*%}"; fi
    if [ "$lib" = new ]; then unset CORDA_AMD_LIB; else export CORDA_AMD_LIB=$PWD/abvar/libcg_$lib.so; fi
    t=${v//[%=]/_}
    env "${envs[@]}" timeout -k 10 200 python -u tools/e2e_sweep.py --pageable-only --sizes $sizes --grid "" \
      --out gpurun_out/$tag/sweep_${t}_$rep.json > gpurun_out/$tag/sweep_${t}_$rep.log 2>&1
  done
done
