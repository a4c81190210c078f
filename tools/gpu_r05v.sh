# round-5 GPU job v: host-buffer verify one past every plan boundary, against the oracle
set -o pipefail
mkdir -p gpurun_out/r05v
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_ed25519.py -k "plan_boundaries" \
  > gpurun_out/r05v/tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r05v/tests.log; exit 1; }
tail -14 gpurun_out/r05v/tests.log
echo done
