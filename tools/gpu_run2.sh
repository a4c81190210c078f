set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload ecdsa --steps 10 --warmup 2 > $O/bench_ecdsa.json 2> $O/bench_ecdsa.err
