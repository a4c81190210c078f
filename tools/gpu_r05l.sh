# round-5 GPU job l: ring chunks staged in 12 MB slices, one-chunk calls through page-locked sliced staging: tests, sweeps
set -o pipefail
mkdir -p gpurun_out/r05l
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_ed25519.py tests/test_gpu_abi.py \
  > gpurun_out/r05l/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05l/tests.log; exit 1; }
tail -3 gpurun_out/r05l/tests.log
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 32 --sizes 4096,65536,262144 --pageable-only --runs 31 --spans --grid ';CORDA_AMD_ONE_PIN=0;CORDA_AMD_ONE_PIN_SLICE_KB=1024;CORDA_AMD_ONE_PIN_SLICE_KB=16384' --out gpurun_out/r05l/e2e_32b.json > gpurun_out/r05l/sweep32.log 2>&1 || exit 2
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 4096,65536 --pageable-only --runs 31 --spans --grid ';CORDA_AMD_ONE_PIN=0;CORDA_AMD_ONE_PIN_SLICE_KB=16384' --out gpurun_out/r05l/e2e_1kb_small.json > gpurun_out/r05l/sweep1ks.log 2>&1 || exit 3
timeout -k 10 500 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 262144,131072 --pageable-only --runs 21 --spans --timeline --grid ';CORDA_AMD_VERIFY_SLICE_KB=0;CORDA_AMD_VERIFY_SLICE_KB=6144;CORDA_AMD_VERIFY_SLICE_KB=24576' --out gpurun_out/r05l/e2e_1kb.json > gpurun_out/r05l/sweep1k.log 2>&1 || exit 4
echo done
