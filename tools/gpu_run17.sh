set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ecdsa.py -x -q --timeout 300 --timeout-method thread > gpurun_out/glv_tests.log 2>&1
