set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile_gpu.sh ${1:?tag} && BENCH_EXTRA="--workload ecdsa --pool 65536" bash tools/profile_gpu.sh ${1}_ecdsa
