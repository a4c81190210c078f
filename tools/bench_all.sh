#!/bin/bash
# Every bench.py workload once, on the GPU box (each under its own time limit):
#   bash tools/bench_all.sh r01n      -> gpurun_out/bench_<tag>_<workload>.json
set -e
TAG=${1:?tag}
mkdir -p gpurun_out
run() {  # workload, extra args
  timeout -k 10 400 python -u bench.py --workload "$1" ${@:2} > gpurun_out/bench_${TAG}_$1.log 2>&1
  tail -1 gpurun_out/bench_${TAG}_$1.log > gpurun_out/bench_${TAG}_$1.json
  echo "$1: $(python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$1.json')); print(d['value'], d['unit'], d['ms_per_step'], 'ms/step')")"
}
run ed25519
run ecdsa --steps 5 --warmup 1
run tx --steps 5 --warmup 1
run ftx --steps 5 --warmup 1
run backlog --steps 2 --warmup 1
