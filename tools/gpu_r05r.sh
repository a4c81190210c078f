# round-5 GPU job r: deferred arena in parts with per-part hash kernels: tests, 1 KB / 32 B sweeps
set -o pipefail
mkdir -p gpurun_out/r05r
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_ed25519.py tests/test_gpu_abi.py \
  > gpurun_out/r05r/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05r/tests.log; exit 1; }
tail -3 gpurun_out/r05r/tests.log
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 4096,16384,65536 --pageable-only --runs 31 --spans --grid ';CORDA_AMD_ARENA_PARTS=1;CORDA_AMD_ARENA_PARTS=3;;CORDA_AMD_ARENA_PARTS=1' --out gpurun_out/r05r/e2e_1kb.json > gpurun_out/r05r/sweep1k.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes 32 --sizes 65536,262144 --pageable-only --runs 31 --spans --grid ';CORDA_AMD_ARENA_PARTS=1' --out gpurun_out/r05r/e2e_32b.json > gpurun_out/r05r/sweep32.log 2>&1 || exit 4
echo done
