# round-6 GPU job g: A/B of the mask selects / branch-free digit abs (ECDSA + Ed25519 MSM), then the bench-layout hash diagnosis (job f)
set -o pipefail
mkdir -p gpurun_out/r06g
AB_REPS=3 AB_ARGS="--workload ecdsa --batch 262144" timeout -k 10 700 bash tools/ab_bench.sh base new || exit 2
mv gpurun_out/ab.txt gpurun_out/r06g/ab_ecdsa.txt
AB_REPS=2 timeout -k 10 400 bash tools/ab_bench.sh base new || exit 3
mv gpurun_out/ab.txt gpurun_out/r06g/ab_ed25519.txt
timeout -k 10 600 bash tools/gpu_r06f.sh || exit 4
echo done
