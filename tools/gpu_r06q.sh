# round-6 GPU job q: whole-call row arrays in the pageable verify pipeline (CG_ROWS_FIRST) — copy-pattern
# ubench, pipeline / mixed-batch GPU tests, then 1 KB e2e A/B against the per-chunk rows (abvar/libcg_perchunk.so)
set -o pipefail
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 200 python -u tools/ubench/h2d_pieces.py --out $O/h2d_pieces.json > $O/h2d_pieces.log 2>&1 || exit 2
timeout -k 10 900 python -u -m pytest tests/test_gpu_ed25519.py tests/test_gpu_ecdsa.py -k "pipeline or plan_boundaries or config2_scale or arena_bounds or all_ed25519 or mixed or host" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 3
for rep in 1 2; do
  for v in new perchunk; do
    if [ $v = new ]; then unset CORDA_AMD_LIB; else export CORDA_AMD_LIB=$PWD/abvar/libcg_perchunk.so; fi
    timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 131073,262144 --pageable-only --runs 21 --grid ';' --spans --bench-layout --out $O/e2e_${v}_$rep.json > $O/e2e_${v}_$rep.log 2>&1 || exit 4
  done
done
unset CORDA_AMD_LIB
echo done
