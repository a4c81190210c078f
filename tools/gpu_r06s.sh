# round-6 GPU job s: ftx pipeline rows in two copies per array (chunk 0's, then every later chunk's) — ftx tests,
# A/B of the ftx workload against the previous library (abvar/libcg_base.so)
set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_merkle.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 2
AB_REPS=2 AB_ARGS="--workload ftx --steps 5 --warmup 1" timeout -k 10 900 bash tools/ab_bench.sh base new > $O/ab.log 2>&1 || exit 3
mv gpurun_out/ab.txt $O/ab_ftx.txt
echo done
