# round-6 GPU job bb: MSM lane-table entries via global instead of flat loads (the select with the shared identity
# entry left a generic pointer), and the same with nontemporal loads — config-2 A/B against the in-tree sources
set -o pipefail
O=gpurun_out/r06bb
mkdir -p $O
AB_REPS=3 timeout -k 10 1000 bash tools/ab_bench.sh base gl glnt > $O/ab.log 2>&1 || exit 2
mv gpurun_out/ab.txt $O/ab_global_loads.txt
echo done
