set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_ed.json 2> $O/bench_ed.err &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-runs 3 --key-reuse 64 > $O/bench_ed_reuse.json 2> $O/bench_ed_reuse.err &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-runs 3 --key-reuse 64 --msg-bytes 32 > $O/bench_ed_reuse32.json 2> $O/bench_ed_reuse32.err &&
bash tools/profile_gpu.sh r02d
