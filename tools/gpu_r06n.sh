# round-6 GPU job n: final-source GPU suite (10 M + 2 M parity inside), smoke, the default driver bench line
set -o pipefail
O=gpurun_out/${TAG:-r06n}
mkdir -p $O
bash tools/gpu_run.sh ${TAG:-r06n} tests smoke || exit 2
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 3
echo done
