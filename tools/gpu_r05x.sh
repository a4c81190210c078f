# round-5 GPU job x: deferred arena from the upload thread beside the row copies: tests, 32 B / 1 KB A/B
set -o pipefail
mkdir -p gpurun_out/r05x
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ed25519.py tests/test_gpu_abi.py \
  > gpurun_out/r05x/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05x/tests.log; exit 1; }
tail -3 gpurun_out/r05x/tests.log
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 32 --sizes 65536,131072,262144 --pageable-only --runs 31 --spans --grid ';CORDA_AMD_ASYNC_ARENA=0;;CORDA_AMD_ASYNC_ARENA=0' --out gpurun_out/r05x/e2e_32b.json > gpurun_out/r05x/sweep32.log 2>&1 || exit 2
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 4096,16384,65536 --pageable-only --runs 31 --spans --grid ';CORDA_AMD_ASYNC_ARENA=0;;CORDA_AMD_ASYNC_ARENA=0' --out gpurun_out/r05x/e2e_1kb.json > gpurun_out/r05x/sweep1k.log 2>&1 || exit 3
echo done
