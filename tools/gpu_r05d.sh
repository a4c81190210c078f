# round-5 GPU job d: host-buffer tests on the new host fast paths, then the 32 B / 1 KB sweeps
set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_ed25519.py tests/test_gpu_abi.py \
  -k "compact or pipeline or one_chunk or latency or reference or abi or golden" > gpurun_out/r05d/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05d/tests.log; exit 1; }
tail -3 gpurun_out/r05d/tests.log
G32=';CORDA_AMD_VERIFY_POLICY=0;CORDA_AMD_VERIFY_CHUNKS=2,CORDA_AMD_VERIFY_MIN_CHUNK=1024,CORDA_AMD_VERIFY_HEAD=0.6,CORDA_AMD_VERIFY_TAIL=1,CORDA_AMD_VERIFY_LANES=0;CORDA_AMD_VERIFY_CHUNKS=2,CORDA_AMD_VERIFY_MIN_CHUNK=1024,CORDA_AMD_VERIFY_HEAD=1,CORDA_AMD_VERIFY_TAIL=1,CORDA_AMD_VERIFY_LANES=0;CORDA_AMD_VERIFY_CHUNKS=3,CORDA_AMD_VERIFY_MIN_CHUNK=1024,CORDA_AMD_VERIFY_HEAD=0.5,CORDA_AMD_VERIFY_TAIL=1,CORDA_AMD_VERIFY_LANES=0'
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 32 --sizes 4096,65536,131072,262144,524288 --pageable-only --runs 21 --spans --grid "$G32" --out gpurun_out/r05d/e2e_32b.json > gpurun_out/r05d/sweep32.log 2>&1 || exit 2
timeout -k 10 400 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 4096,65536,262144 --pageable-only --runs 21 --spans --grid ';CORDA_AMD_VERIFY_POLICY=0' --out gpurun_out/r05d/e2e_1kb.json > gpurun_out/r05d/sweep1k.log 2>&1 || exit 3
echo done
