# full GPU suite + every bench workload (+ the key-reuse / 32 B variants) on the current kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:?tag}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 && \
bash tools/bench_all.sh $TAG && \
timeout -k 10 300 python -u bench.py --key-reuse 64 > gpurun_out/bench_${TAG}_ed25519_reuse64.log 2>&1 && \
timeout -k 10 300 python -u bench.py --msg-bytes 32 > gpurun_out/bench_${TAG}_ed25519_32b.log 2>&1
