# round-5 GPU job aa: byte-aware latency-mode threshold for one-chunk calls (32 B 20,480; 1 KB 32,768)
set -o pipefail
mkdir -p gpurun_out/r05aa
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ed25519.py tests/test_gpu_abi.py \
  > gpurun_out/r05aa/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05aa/tests.log; exit 1; }
tail -3 gpurun_out/r05aa/tests.log
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 32 --sizes 16384,24576,32768,40000 --pageable-only --runs 31 --grid ';CORDA_AMD_ED_PAIR_MAX=40000' --out gpurun_out/r05aa/e2e_32b.json > gpurun_out/r05aa/sweep32.log 2>&1 || exit 2
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 16384,32768,40000 --pageable-only --runs 31 --grid ';CORDA_AMD_ED_PAIR_MAX=40000' --out gpurun_out/r05aa/e2e_1kb.json > gpurun_out/r05aa/sweep1k.log 2>&1 || exit 3
echo done
