# north-star parity on the current kernels: 10 M Ed25519 + 2 M ECDSA adversarial mixes vs the C
# restatement, both modes; then the tx chunk sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CORDA_AMD_PARITY_N=10000000 CORDA_AMD_PARITY_EC_N=2097152 timeout -k 10 800 python -u -m pytest tests/test_gpu_parity_mix.py -s -q --timeout 780 --timeout-method thread > gpurun_out/${1:-r02v}_parity_big.txt 2>&1 && \
rm -rf gpurun_out/txc && bash tools/tx_chunks.sh 4 6 8 10 12
