# round-5 GPU job w: split points (key half beside the signature rows' copy): tests, 32 B A/B
set -o pipefail
mkdir -p gpurun_out/r05w
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ed25519.py tests/test_gpu_abi.py \
  > gpurun_out/r05w/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05w/tests.log; exit 1; }
tail -3 gpurun_out/r05w/tests.log
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 32 --sizes 50000,65536,131072 --pageable-only --runs 31 --spans --grid ';CORDA_AMD_SPLIT_POINTS=0;;CORDA_AMD_SPLIT_POINTS=0' --out gpurun_out/r05w/e2e_32b.json > gpurun_out/r05w/sweep32.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 65536 --pageable-only --runs 21 --spans --grid ';CORDA_AMD_SPLIT_POINTS=0' --out gpurun_out/r05w/e2e_1kb.json > gpurun_out/r05w/sweep1k.log 2>&1 || exit 3
echo done
