# final evidence of a kernel-source state: PMC passes (Ed25519, ECDSA, key-reuse) + bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:?tag}
bash tools/profile_gpu.sh $T && BENCH_EXTRA="--workload ecdsa --pool 65536" bash tools/profile_gpu.sh ${T}_ecdsa && \
BENCH_EXTRA="--key-reuse 64" bash tools/profile_gpu.sh ${T}_reuse
