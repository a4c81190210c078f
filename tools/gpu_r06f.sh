# round-6 GPU job f: which part of the bench layout slows the hash kernel (65,536 / 262,144 x 32 B)
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
S="--msg-bytes 32 --sizes 65536,262144 --pageable-only --runs 21 --grid ; --spans"
run() { timeout -k 10 300 python -u tools/e2e_sweep.py $S --out $O/$1.json "${@:2}" > $O/$1.log 2>&1; }
run valid && run ragged --force-ragged && run adv_all --bench-layout && run adv_E12 --bench-layout --adv-classes E12 \
 && run adv_E1_E6 --bench-layout --adv-classes E1,E2,E3,E4,E5,E6 && run adv_E7_E11 --bench-layout --adv-classes E7,E8,E9,E10,E11 || exit 2
echo done
