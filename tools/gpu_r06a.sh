# round-6 GPU job a: exact digit counts + grouped MSM — parity, then config-2 A/B (grouping on / off)
set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 600 python -u -m pytest tests/test_gpu_ed25519.py -x -v --timeout 300 --timeout-method thread -k "grouped or golden or random_and_mutated or forced_full or latency_mode or config2_scale" > gpurun_out/r06a/tests.log 2>&1 || exit 2
for v in on off on off; do
  if [ $v = off ]; then export CORDA_AMD_ED_BUCKET_MIN=0; else unset CORDA_AMD_ED_BUCKET_MIN; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline --latency-runs 3 > gpurun_out/r06a/bench_$v.json 2>> gpurun_out/r06a/bench.err || exit 3
  cat gpurun_out/r06a/bench_$v.json >> gpurun_out/r06a/bench_all.jsonl
done
echo done
