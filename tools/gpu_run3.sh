set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ed25519.py -x -v --timeout 300 --timeout-method thread > $O/gpu_ed.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-runs 3 > $O/bench_ed.json 2> $O/bench_ed.err &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-runs 3 --key-reuse 64 > $O/bench_ed_reuse.json 2> $O/bench_ed_reuse.err &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-runs 3 --key-reuse 64 --msg-bytes 32 > $O/bench_ed_reuse32.json 2> $O/bench_ed_reuse32.err
