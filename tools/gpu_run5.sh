set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02e; mkdir -p $O
timeout -k 10 300 python -u bench.py --workload tx --steps 5 --warmup 2 > $O/bench_tx.json 2> $O/bench_tx.err &&
timeout -k 10 300 python -u bench.py --workload tx --steps 5 --warmup 2 --no-cpu-baseline --key-reuse 256 > $O/bench_tx_reuse.json 2> $O/bench_tx_reuse.err &&
timeout -k 10 400 python -u bench.py --workload backlog --steps 3 --warmup 1 --key-reuse 64 > $O/bench_backlog_reuse.json 2> $O/bench_backlog_reuse.err &&
BENCH_EXTRA="--workload ecdsa --pool 65536" bash tools/profile_gpu.sh r02e_ecdsa
