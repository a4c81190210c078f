# round-5 GPU job e: deferred offsets/lengths + parallel arena scan: host-buffer tests, sweeps, full bench line
set -o pipefail
mkdir -p gpurun_out/r05e
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_ed25519.py tests/test_gpu_abi.py tests/test_gpu_signatures.py \
  > gpurun_out/r05e/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05e/tests.log; exit 1; }
tail -3 gpurun_out/r05e/tests.log
timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes 32 --sizes 4096,65536,262144 --pageable-only --runs 21 --spans --grid ';CORDA_AMD_VERIFY_POLICY=0' --out gpurun_out/r05e/e2e_32b.json > gpurun_out/r05e/sweep32.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 4096,65536,262144 --pageable-only --runs 21 --spans --grid ';CORDA_AMD_VERIFY_TAIL=0.25' --out gpurun_out/r05e/e2e_1kb.json > gpurun_out/r05e/sweep1k.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r05e/bench.log 2>&1 || { tail -20 gpurun_out/r05e/bench.log; exit 4; }
tail -1 gpurun_out/r05e/bench.log > gpurun_out/r05e/bench_ed25519.json
echo done
