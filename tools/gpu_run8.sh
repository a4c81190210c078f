set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02n; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_merkle.py > $O/tests.log 2>&1 || exit 1
CORDA_AMD_TIMELINE=$O/timeline_k8.txt timeout -k 10 300 python -u bench.py --workload tx --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_tx_tl.json 2> $O/bench_tx_tl.err &&
for K in 4 6 8; do
  CORDA_AMD_TX_CHUNKS=$K CORDA_AMD_TX_MIN_CHUNK=32768 timeout -k 10 300 python -u bench.py --workload tx --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_tx_k$K.json 2> $O/bench_tx_k$K.err || exit 1
done
timeout -k 10 300 python -u bench.py --workload ecdsa --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_ecdsa.json 2> $O/bench_ecdsa.err &&
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_ed.json 2> $O/bench_ed.err
