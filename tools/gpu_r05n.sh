# round-5 GPU job n: pageable copies from a helper thread (RING=2) against the ring: pipeline tests, 1 KB sweep
set -o pipefail
mkdir -p gpurun_out/r05n
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_ed25519.py -k "small_chunks or pipeline or compute_bound" \
  > gpurun_out/r05n/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05n/tests.log; exit 1; }
tail -3 gpurun_out/r05n/tests.log
timeout -k 10 600 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 262144,131072 --pageable-only --runs 21 --spans --timeline --grid ';CORDA_AMD_VERIFY_RING=2;CORDA_AMD_VERIFY_RING=0;;CORDA_AMD_VERIFY_RING=2' --out gpurun_out/r05n/e2e_1kb.json > gpurun_out/r05n/sweep1k.log 2>&1 || exit 4
echo done
