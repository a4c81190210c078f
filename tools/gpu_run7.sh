set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02h; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_merkle.py > $O/tests.log 2>&1 || exit 1
for K in 3 4 5 6 8; do
  CORDA_AMD_TX_CHUNKS=$K CORDA_AMD_TX_MIN_CHUNK=32768 timeout -k 10 300 python -u bench.py --workload tx --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_tx_k$K.json 2> $O/bench_tx_k$K.err || exit 1
done
CORDA_AMD_TX_CHUNKS=5 CORDA_AMD_TX_MIN_CHUNK=32768 timeout -k 10 300 python -u bench.py --workload tx --steps 5 --warmup 2 --no-cpu-baseline --key-reuse 256 > $O/bench_tx_reuse_k5.json 2> $O/bench_tx_reuse_k5.err
