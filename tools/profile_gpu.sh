#!/bin/bash
# Kernel trace + PMC passes over a short bench run, on the GPU box:
#   bash tools/profile_gpu.sh r02d              (BENCH_EXTRA="--workload ecdsa" for config 3)
# Each rocprofv3 pass runs alone under its own time limit (counters are never
# combined with runtime/sys traces; <= 8 SQ and <= 4 TCC counters per pass).
# Outputs: gpurun_out/prof_<tag>/ ; reduce with tools/pmc_report.py here.
set -e
TAG=${1:?tag}
export TMPDIR=/tmp
# every launch alone on the GPU (no points kernel beside the hash kernel), so the trace's
# per-kernel durations are the isolated ones the bench's `kernels` table reports
export CORDA_AMD_ED_OVERLAP=0
O=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p "$O"
ARGS="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --latency-runs 1 ${BENCH_EXTRA:-}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o trace -- python3 $ARGS > "$O/trace.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d "$O/p1" -o p1 -- python3 $ARGS > "$O/p1.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VALU_INT64 GRBM_COUNT --output-format csv -d "$O/p2" -o p2 -- python3 $ARGS > "$O/p2.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/p3" -o p3 -- python3 $ARGS > "$O/p3.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/p4" -o p4 -- python3 $ARGS > "$O/p4.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$O/p5" -o p5 -- python3 $ARGS > "$O/p5.log" 2>&1
find "$O" -name "*.csv" | sort
