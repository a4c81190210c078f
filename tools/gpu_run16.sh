# PMC passes of the key-reuse path (64 signers): cg_ed25519_points_r / msm_r / keyprep
set -o pipefail
cd $GRAFT_REPO_ROOT
BENCH_EXTRA="--key-reuse 64" bash tools/profile_gpu.sh ${1:?tag}_reuse
