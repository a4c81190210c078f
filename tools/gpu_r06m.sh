# round-6 GPU job m: limb doublings as 2-cycle v_add_u32 (Ed25519 prescales, P-256 / secp256k1 prescales and
# formula doublings) — Ed25519 + ECDSA GPU tests, then A/B against the previous library (abvar/libcg_base.so)
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_ed25519.py tests/test_gpu_ecdsa.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 2
AB_REPS=3 timeout -k 10 700 bash tools/ab_bench.sh base new > $O/ab_ed.log 2>&1 || exit 3
mv gpurun_out/ab.txt $O/ab_ed25519.txt
AB_REPS=2 AB_ARGS="--workload ecdsa" timeout -k 10 700 bash tools/ab_bench.sh base new > $O/ab_ec.log 2>&1 || exit 4
mv gpurun_out/ab.txt $O/ab_ecdsa.txt
echo done
