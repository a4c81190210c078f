# round-6 GPU job aa: pipeline chunks >= 2 start their staging and points kernels on the whole-call rows (ev[1])
# and only their arena's readers wait for the chunk's copy — pipeline GPU tests, host-ASan driver, 1 KB e2e A/B
set -o pipefail
O=gpurun_out/r06aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_abi.py tests/test_gpu_ed25519.py tests/test_gpu_ecdsa.py -k "native or asan or pipeline or plan_boundaries or config2_scale or mixed or host or all_ed25519 or arena" -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || exit 2
for rep in 1 2; do
  for v in new base; do
    if [ $v = new ]; then unset CORDA_AMD_LIB; else export CORDA_AMD_LIB=$PWD/abvar/libcg_$v.so; fi
    timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes 1024 --sizes 131073,262144,393216 --pageable-only --runs 21 --grid ';' --spans --bench-layout --out $O/e2e_${v}_$rep.json > $O/e2e_${v}_$rep.log 2>&1 || exit 3
  done
done
unset CORDA_AMD_LIB
echo done
