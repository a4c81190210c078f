# round-5 GPU job m: A/B on one box: one-chunk page-locked staging on/off; ring slices / no ring at 2^17..2^18 x 1 KB
set -o pipefail
mkdir -p gpurun_out/r05m
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 32 --sizes 65536,262144 --pageable-only --runs 31 --spans --grid ';CORDA_AMD_ONE_PIN=0;;CORDA_AMD_ONE_PIN=0' --out gpurun_out/r05m/e2e_32b.json > gpurun_out/r05m/sweep32.log 2>&1 || exit 2
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 4096,65536 --pageable-only --runs 31 --spans --grid ';CORDA_AMD_ONE_PIN=0;;CORDA_AMD_ONE_PIN=0' --out gpurun_out/r05m/e2e_1kb_small.json > gpurun_out/r05m/sweep1ks.log 2>&1 || exit 3
timeout -k 10 500 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 262144 --pageable-only --runs 21 --spans --timeline --grid ';CORDA_AMD_VERIFY_SLICE_KB=0;CORDA_AMD_VERIFY_RING=0;;CORDA_AMD_VERIFY_SLICE_KB=0;CORDA_AMD_VERIFY_RING=0' --out gpurun_out/r05m/e2e_1kb.json > gpurun_out/r05m/sweep1k.log 2>&1 || exit 4
echo done
