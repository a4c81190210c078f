# round-6 GPU job dd: PMC + trace passes on the final sources (global table loads), then the default driver line
set -o pipefail
O=gpurun_out/r06dd
mkdir -p $O
bash tools/gpu_run.sh r06dd profile=ed profile=ec:--workload:ecdsa:--batch:524288 profile=reuse:--key-reuse:64 || exit 3
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 4
echo done
