# round-5 GPU job s: pipeline error / allocation-failure recovery under the upload thread
set -o pipefail
mkdir -p gpurun_out/r05s
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_ed25519.py -k "errors_then_recovery or small_chunks" \
  > gpurun_out/r05s/tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r05s/tests.log; exit 1; }
tail -3 gpurun_out/r05s/tests.log
echo done
