# round-6 GPU job e: end to end on the driver bench line's layout vs the valid-only layout, with spans
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
for mb in 32 1024; do
  timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes $mb --sizes 4096,65536,262144 --pageable-only --runs 31 --grid ';' --spans --bench-layout --out $O/bench_layout_$mb.json > $O/bench_layout_$mb.log 2>&1 || exit 2
  timeout -k 10 300 python -u tools/e2e_sweep.py --msg-bytes $mb --sizes 4096,65536,262144 --pageable-only --runs 31 --grid ';' --spans --out $O/valid_$mb.json > $O/valid_$mb.log 2>&1 || exit 3
done
echo done
