# round-6 GPU job v: async arena for 1-8 MB arenas of one-chunk calls >= 32,768 (the upload thread is awake
# with the bounds pass) — 32 B e2e A/B at the bench layout against the in-tree library
set -o pipefail
O=gpurun_out/r06v
mkdir -p $O
for rep in 1 2; do
  for v in new a1m; do
    if [ $v = new ]; then unset CORDA_AMD_LIB; else export CORDA_AMD_LIB=$PWD/abvar/libcg_$v.so; fi
    timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes 32 --sizes 40001,65536,100000 --pageable-only --runs 31 --grid ';' --spans --bench-layout --out $O/e2e_${v}_$rep.json > $O/e2e_${v}_$rep.log 2>&1 || exit 2
  done
done
unset CORDA_AMD_LIB
echo done
