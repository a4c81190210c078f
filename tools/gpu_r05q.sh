# round-5 GPU job q: runtime pageable copies from the persistent upload thread (default), ring as option: tests, 1 KB sweep
set -o pipefail
mkdir -p gpurun_out/r05q
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_ed25519.py tests/test_gpu_abi.py tests/test_gpu_signatures.py \
  > gpurun_out/r05q/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05q/tests.log; exit 1; }
tail -3 gpurun_out/r05q/tests.log
timeout -k 10 600 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 262144,131072,65536,4096 --pageable-only --runs 21 --spans --timeline --grid ';CORDA_AMD_VERIFY_RING=1;CORDA_AMD_VERIFY_TAIL=0.17;CORDA_AMD_VERIFY_TAIL=0.35;' --out gpurun_out/r05q/e2e_1kb.json > gpurun_out/r05q/sweep1k.log 2>&1 || exit 4
echo done
