set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02f; mkdir -p $O
for K in 4 8 12 16; do
  CORDA_AMD_TX_CHUNKS=$K CORDA_AMD_TX_MIN_CHUNK=32768 timeout -k 10 300 python -u bench.py --workload tx --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_tx_k$K.json 2> $O/bench_tx_k$K.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -- python3 bench.py --workload tx --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
