# round-6 GPU job h: automaton slide carry + late S load (hash kernel: no spills) — Ed25519 GPU suite, A/B vs base, e2e bench layout
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_ed25519.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 2
AB_REPS=2 timeout -k 10 400 bash tools/ab_bench.sh base new || exit 3
mv gpurun_out/ab.txt $O/ab_ed25519.txt
for mb in 32 1024; do
  timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes $mb --sizes 4096,65536,262144 --pageable-only --runs 31 --grid ';' --spans --bench-layout --out $O/bench_layout_$mb.json > $O/bench_layout_$mb.log 2>&1 || exit 4
done
echo done
