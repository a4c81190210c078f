# round-6 GPU job r: pipeline tail / chunk count once per-chunk row copies are gone (1 KB, bench layout)
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
G=';CORDA_AMD_VERIFY_TAIL=0.15;CORDA_AMD_VERIFY_TAIL=0.1;CORDA_AMD_VERIFY_CHUNKS=12;CORDA_AMD_VERIFY_CHUNKS=12,CORDA_AMD_VERIFY_TAIL=0.15;CORDA_AMD_VERIFY_HEAD=0.15'
for rep in 1 2; do
  timeout -k 10 500 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 131073,262144,393216 --pageable-only --runs 21 --grid "$G" --spans --bench-layout --out $O/grid_$rep.json > $O/grid_$rep.log 2>&1 || exit 2
done
echo done
