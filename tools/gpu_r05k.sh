# round-5 GPU job k: sliced ring staging of the first two chunks, tail taper: pipeline tests, 1 KB sweep + timeline
set -o pipefail
mkdir -p gpurun_out/r05k
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_ed25519.py tests/test_gpu_abi.py -k "small_chunks" \
  > gpurun_out/r05k/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05k/tests.log; exit 1; }
tail -3 gpurun_out/r05k/tests.log
timeout -k 10 500 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 262144,131072 --pageable-only --runs 21 --spans --timeline --grid ';CORDA_AMD_VERIFY_SLICES=1;CORDA_AMD_VERIFY_SLICES=8;CORDA_AMD_VERIFY_TAPER=0.5:0.25;CORDA_AMD_VERIFY_TAPER=0.5:0.25:0.125;CORDA_AMD_VERIFY_TAPER=0.6:0.3:0.15,CORDA_AMD_VERIFY_CHUNKS=10,CORDA_AMD_VERIFY_MIN_CHUNK=24000;' --out gpurun_out/r05k/e2e_1kb.json > gpurun_out/r05k/sweep1k.log 2>&1 || exit 3
echo done
