# round-6 GPU job l: arena-bounds pass beside the row copies — its tests, then e2e at the bench layout
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ed25519.py -k "arena_bounds or plan_boundaries or pipeline_errors" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 2
for mb in 32 1024; do
  timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes $mb --sizes 4096,65536,262144 --pageable-only --runs 31 --grid ';' --spans --bench-layout --out $O/bench_layout_$mb.json > $O/bench_layout_$mb.log 2>&1 || exit 4
done
timeout -k 10 400 python -u tools/e2e_pattern.py --rounds 2 --out $O/pattern.json > $O/pattern.log 2>&1 || exit 5
echo done
