# round-5 GPU job z: latency-mode threshold against balanced + split points at 16k-40k signatures
set -o pipefail
mkdir -p gpurun_out/r05z
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 32 --sizes 16384,24576,32768,40000 --pageable-only --runs 31 --grid ';CORDA_AMD_ED_PAIR_MAX=12000;;CORDA_AMD_ED_PAIR_MAX=12000' --out gpurun_out/r05z/e2e_32b.json > gpurun_out/r05z/sweep32.log 2>&1 || exit 2
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 16384,24576,32768,40000 --pageable-only --runs 31 --grid ';CORDA_AMD_ED_PAIR_MAX=12000;;CORDA_AMD_ED_PAIR_MAX=12000' --out gpurun_out/r05z/e2e_1kb.json > gpurun_out/r05z/sweep1k.log 2>&1 || exit 3
echo done
