# round-6 GPU job i: config-2 step plan A/B on the spill-free hash kernel: points beside hash (default) / after it / two pieces
set -o pipefail
mkdir -p gpurun_out/r06i
AB_REPS=3 timeout -k 10 900 bash tools/ab_bench.sh new new%CORDA_AMD_ED_OVERLAP=0 new%CORDA_AMD_ED_SPLIT=2 || exit 2
mv gpurun_out/ab.txt gpurun_out/r06i/ab_step_plan.txt
echo done
