# round-6 GPU job t: MSM occupancy A/B — 3 waves/SIMD (168 VGPRs, spills: Ed25519 13, K1 15, R1 62) vs 2
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
AB_REPS=3 timeout -k 10 700 bash tools/ab_bench.sh base w3 > $O/ab_ed.log 2>&1 || exit 2
mv gpurun_out/ab.txt $O/ab_ed25519.txt
AB_REPS=2 AB_ARGS="--workload ecdsa" timeout -k 10 700 bash tools/ab_bench.sh base w3 > $O/ab_ec.log 2>&1 || exit 3
mv gpurun_out/ab.txt $O/ab_ecdsa.txt
echo done
