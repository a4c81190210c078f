# round-6 GPU job b: grouped MSM (two-pass, no atomics) — parity, trace + VALU PMC with grouping on / off, A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ed25519.py -x -v --timeout 300 --timeout-method thread -k "grouped or golden" > $O/tests.log 2>&1 || exit 2
ARGS="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --latency-runs 1"
export CORDA_AMD_ED_OVERLAP=0
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_on -o trace -- python3 $ARGS > $O/trace_on.log 2>&1 || exit 3
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p1_on -o p1 -- python3 $ARGS > $O/p1_on.log 2>&1 || exit 4
export CORDA_AMD_ED_BUCKET_MIN=0
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p1_off -o p1 -- python3 $ARGS > $O/p1_off.log 2>&1 || exit 5
unset CORDA_AMD_ED_OVERLAP
for v in on off on off; do
  if [ $v = off ]; then export CORDA_AMD_ED_BUCKET_MIN=0; else unset CORDA_AMD_ED_BUCKET_MIN; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline --latency-runs 3 > $O/bench_$v.json 2>> $O/bench.err || exit 6
  cat $O/bench_$v.json >> $O/bench_all.jsonl
done
echo done
