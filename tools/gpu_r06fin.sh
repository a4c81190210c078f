# round-6 final GPU job: default driver bench line, every workload's line, e2e at the bench layout
set -o pipefail
O=gpurun_out/r06fin
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 2
bash tools/gpu_run.sh r06fin benchall || exit 3
for mb in 32 1024; do
  timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes $mb --sizes 4096,65536,262144 --pageable-only --runs 31 --grid ';' --spans --bench-layout --out $O/bench_layout_$mb.json > $O/bench_layout_$mb.log 2>&1 || exit 4
done
echo done
