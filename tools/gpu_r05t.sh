# round-5 GPU job t: latency lanes for the whole chunks of a copy-bound pipeline (2^17-2^18 x 1 KB)
set -o pipefail
mkdir -p gpurun_out/r05t
timeout -k 10 600 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 262144,131072 --pageable-only --runs 21 --spans --timeline --grid ';CORDA_AMD_ED_PAIR_MAX=45000;CORDA_AMD_ED_PAIR_MAX=45000,CORDA_AMD_ED_QUAD_MAX=45000;;CORDA_AMD_ED_PAIR_MAX=45000' --out gpurun_out/r05t/e2e_1kb.json > gpurun_out/r05t/sweep1k.log 2>&1 || exit 3
echo done
