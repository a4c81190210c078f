# round-6 GPU job d: options snapshot (cg_set_option) + host plan refactor — Ed25519 / Merkle / ABI / dist GPU suites, smoke, bench
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_ed25519.py tests/test_gpu_merkle.py tests/test_gpu_abi.py tests/test_gpu_signatures.py tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline --latency-runs 11 > $O/bench.json 2> $O/bench.err || exit 4
echo done
