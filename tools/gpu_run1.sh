set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02a
timeout -k 10 120 ./tools/ubench/isa_rates > gpurun_out/r02a/isa_rates.json 2> gpurun_out/r02a/isa_rates.err &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/r02a/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r02a/bench.json 2> gpurun_out/r02a/bench.err
