# round-6 GPU job c: the driver's default bench line (config 2 + 32 B e2e + full config 3 + config 4), timed
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
SECONDS=0; timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 2; echo "wall_s=$SECONDS" >> $O/bench.err
echo done
