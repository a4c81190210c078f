# round-5 GPU job u: latency lanes for the last two chunks of a copy-bound pipeline: tests, 1 KB sweep
set -o pipefail
mkdir -p gpurun_out/r05u
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_ed25519.py -k "small_chunks or pipeline or recovery" \
  > gpurun_out/r05u/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05u/tests.log; exit 1; }
tail -3 gpurun_out/r05u/tests.log
timeout -k 10 600 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 262144,131072,196608,393216 --pageable-only --runs 21 --spans --grid ';CORDA_AMD_PIPE_TAIL_PAIR=0;;CORDA_AMD_PIPE_TAIL_PAIR=0' --out gpurun_out/r05u/e2e_1kb.json > gpurun_out/r05u/sweep1k.log 2>&1 || exit 3
echo done
