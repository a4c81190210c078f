# round-6 GPU job ff: SHA message words via global instead of flat loads (the 4-byte-aligned base pointer was
# rebuilt from an integer, losing its address space) — config-2 A/B against the in-tree library
set -o pipefail
O=gpurun_out/r06ff
mkdir -p $O
AB_REPS=3 timeout -k 10 900 bash tools/ab_bench.sh base hg > $O/ab.log 2>&1 || exit 2
mv gpurun_out/ab.txt $O/ab_hash_global.txt
echo done
