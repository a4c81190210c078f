# round-6 GPU job z: copy-bound pipeline chunks in the two-lane latency mode (CORDA_AMD_ED_PAIR_MAX above the
# regular chunk size) — 1 KB e2e at the bench layout
set -o pipefail
O=gpurun_out/r06z
mkdir -p $O
G=';CORDA_AMD_ED_PAIR_MAX=65536;CORDA_AMD_ED_PAIR_MAX=65536,CORDA_AMD_VERIFY_CHUNKS=6'
for rep in 1 2; do
  timeout -k 10 500 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 131073,196608,262144,393216 --pageable-only --runs 21 --grid "$G" --spans --bench-layout --out $O/grid_$rep.json > $O/grid_$rep.log 2>&1 || exit 2
done
echo done
