set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02p; mkdir -p $O
CORDA_AMD_TIMELINE=$O/timeline.txt timeout -k 10 300 python -u bench.py --workload tx --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_tx_tl.json 2> $O/bench_tx_tl.err &&
for K in 4 6 8; do
  CORDA_AMD_TX_CHUNKS=$K CORDA_AMD_TX_MIN_CHUNK=32768 timeout -k 10 300 python -u bench.py --workload tx --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_tx_k$K.json 2> $O/bench_tx_k$K.err || exit 1
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_ed.json 2> $O/bench_ed.err &&
timeout -k 10 300 python -u bench.py --workload ecdsa --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_ecdsa.json 2> $O/bench_ecdsa.err
