# bench lines of every workload on the current tree -> gpurun_out/bench_<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:?tag}
O=gpurun_out/bench_$T; mkdir -p $O
b() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim python -u bench.py "$@" > $O/$name.json 2> $O/$name.err; }
b ed25519 300 && b ed25519_32b 300 --msg-bytes 32 && b ed25519_reuse64 300 --key-reuse 64 --no-cpu-baseline && \
b ecdsa 300 --workload ecdsa && b tx 300 --workload tx --steps 5 --warmup 2 && \
b ftx 300 --workload ftx --steps 5 --warmup 1 && b backlog 500 --workload backlog --steps 2 --warmup 1
