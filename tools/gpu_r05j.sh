# round-5 GPU job j: lane modes at 65,536 x 32 B; 262,144 x 1 KB per-span timeline
set -o pipefail
mkdir -p gpurun_out/r05j
timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes 32 --sizes 65536 --pageable-only --runs 41 --spans --grid ';CORDA_AMD_ED_PAIR_MAX=70000;CORDA_AMD_ED_PAIR_MAX=70000,CORDA_AMD_ED_QUAD_MAX=70000;' --out gpurun_out/r05j/e2e_32b.json > gpurun_out/r05j/sweep32.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 262144 --pageable-only --runs 21 --spans --timeline --grid ';' --out gpurun_out/r05j/e2e_1kb.json > gpurun_out/r05j/sweep1k.log 2>&1 || exit 3
echo done
