# round-5 GPU job h: early points in >= 65,536 parts, raw rows for the balanced points kernel: tests, 32 B A/B
set -o pipefail
mkdir -p gpurun_out/r05h
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_ed25519.py tests/test_gpu_abi.py \
  > gpurun_out/r05h/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05h/tests.log; exit 1; }
tail -3 gpurun_out/r05h/tests.log
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 32 --sizes 65536,131072,262144 --pageable-only --runs 21 --spans --grid ';CORDA_AMD_EARLY_POINTS=0;CORDA_AMD_EARLY_POINTS=2' --out gpurun_out/r05h/e2e_32b.json > gpurun_out/r05h/sweep32.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 4096,65536,262144 --pageable-only --runs 21 --spans --grid ';' --out gpurun_out/r05h/e2e_1kb.json > gpurun_out/r05h/sweep1k.log 2>&1 || exit 3
echo done
