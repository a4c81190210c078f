# round-5 GPU job f: compute-bound pipeline variants (uploads one chunk ahead), fused points+MSM A/B
set -o pipefail
mkdir -p gpurun_out/r05f
P='CORDA_AMD_VERIFY_MIN_CHUNK=1024,CORDA_AMD_VERIFY_LANES=0,CORDA_AMD_VERIFY_AHEAD=1'
G=";CORDA_AMD_VERIFY_CHUNKS=2,CORDA_AMD_VERIFY_HEAD=0.5,CORDA_AMD_VERIFY_TAIL=1,$P;CORDA_AMD_VERIFY_CHUNKS=2,CORDA_AMD_VERIFY_HEAD=0.3,CORDA_AMD_VERIFY_TAIL=1,$P;CORDA_AMD_VERIFY_CHUNKS=3,CORDA_AMD_VERIFY_HEAD=0.5,CORDA_AMD_VERIFY_TAIL=1,$P;CORDA_AMD_VERIFY_CHUNKS=4,CORDA_AMD_VERIFY_HEAD=0.5,CORDA_AMD_VERIFY_TAIL=1,$P;CORDA_AMD_VERIFY_CHUNKS=2,CORDA_AMD_VERIFY_HEAD=0.5,CORDA_AMD_VERIFY_TAIL=1,$P,CORDA_AMD_VERIFY_RING=0"
timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes 32 --sizes 65536,262144,524288 --pageable-only --runs 21 --spans --grid "$G" --out gpurun_out/r05f/e2e_32b.json > gpurun_out/r05f/sweep32.log 2>&1 || exit 2
AB_REPS=2 timeout -k 10 500 bash tools/ab_bench.sh new new%CORDA_AMD_ED_FUSE=1 > gpurun_out/r05f/ab.log 2>&1 || exit 3
cp gpurun_out/ab.txt gpurun_out/r05f/ab.txt; cat gpurun_out/r05f/ab.txt
echo done
