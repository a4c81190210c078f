# round-6 GPU job: timing probe (wrong verdicts, never a product build) — every MSM lane reads one of 64 lane
# tables, so the table reads hit L2: what the MSM's table traffic costs on the round-6 kernels
set -o pipefail
O=gpurun_out/r06probe
mkdir -p $O
AB_REPS=3 timeout -k 10 700 bash tools/ab_bench.sh new ${AB_VARIANT:-fake} > $O/ab.log 2>&1 || exit 2
mv gpurun_out/ab.txt $O/ab_${AB_VARIANT:-fake}_table.txt
echo done
