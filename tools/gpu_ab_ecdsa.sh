# GPU parity (ECDSA suites) of the in-tree library, then A/B timing of config 3 vs abvar/ variants
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ecdsa.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_gpu_tests.log 2>&1 && \
rm -f gpurun_out/ab.txt && AB_ARGS="--workload ecdsa" bash tools/ab_bench.sh ${AB_NAMES:-prev new}
