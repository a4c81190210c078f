# round-6 GPU job w: final host plan — plan / bounds / scheme-array GPU tests, PMC passes on the final sources
# (the plan header is part of the kernel-source hash), the default driver bench line
set -o pipefail
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ed25519.py -k "plan_boundaries or arena_bounds or all_ed25519 or options or latency or pipeline" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 2
bash tools/gpu_run.sh r06w profile=ed profile=ec:--workload:ecdsa:--batch:524288 profile=reuse:--key-reuse:64 || exit 3
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 4
echo done
