set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python3 bench.py --workload tx --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
