#!/bin/bash
# One parameterised GPU-box runner (replaces the per-round gpu_runN.sh scripts):
#
#   bash tools/gpu_run.sh <tag> <step> [<step> ...]
#
# Steps run in order, each under its own time limit, and the first failure ends the
# run (nothing more touches the GPU after a fault, abort or timeout).  Outputs go to
# gpurun_out/<tag>/.  Steps:
#   tests[=<pytest args>]     pytest -m gpu (default: the whole GPU suite)     tests.log
#   smoke                     __graft_entry__.smoke()                           smoke.log
#   bench=<name>[:<args>]     python bench.py <args> (':' separates args)      bench_<name>.json / .err
#   benchall                  every workload's bench line (config 2, 32 B ids, 64 signers,
#                             config 3, config 4, ftx, config 5)                bench_<workload>.json
#   profile=<name>[:<args>]   rocprofv3 trace + PMC passes of bench.py <args>   prof_<name>/
#   parity=<n>[:<n_ec>]       tests/test_gpu_parity_mix.py at n Ed25519 / n_ec ECDSA  parity.log
#   ab=<variants>[@<args>]    tools/ab_bench.sh over abvar/ variants (':' separated), bench args
#                             after '@' (':' separated)                           ab_<tag>.txt
# Example:
#   gpurun --timeout 1200 -- 'bash tools/gpu_run.sh r03a tests smoke bench=ed25519 profile=ed:'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${1:?usage: gpu_run.sh <tag> <step>...}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp

args_of() { echo "${1//:/ }"; }

run_step() {
  local step=$1 name=${1%%=*} val=
  [[ $step == *=* ]] && val=${step#*=}
  echo "== $step ($(date +%T))"
  case $name in
    tests)
      timeout -k 10 900 python -u -m pytest ${val:-tests -m gpu} -x -v --timeout 300 --timeout-method thread \
        > "$O/tests.log" 2>&1 ;;
    smoke)
      timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    bench)
      local b=${val%%:*} a=
      [[ $val == *:* ]] && a=$(args_of "${val#*:}")
      timeout -k 10 600 python -u bench.py $a > "$O/bench_$b.json" 2> "$O/bench_$b.err" ;;
    benchall)
      run_step "bench=ed25519" && run_step "bench=ed25519_32b:--msg-bytes:32:--no-cpu-baseline" && \
      run_step "bench=ed25519_reuse64:--key-reuse:64:--no-cpu-baseline" && \
      run_step "bench=ecdsa:--workload:ecdsa" && run_step "bench=tx:--workload:tx:--steps:5:--warmup:2" && \
      run_step "bench=ftx:--workload:ftx:--steps:5:--warmup:1" && \
      run_step "bench=backlog:--workload:backlog:--steps:2:--warmup:1" ;;
    profile)
      local p=${val%%:*} a=
      [[ $val == *:* ]] && a=$(args_of "${val#*:}")
      BENCH_EXTRA="$a" bash tools/profile_gpu.sh "${TAG}_$p" > "$O/profile_$p.log" 2>&1 ;;
    parity)
      local ne=${val%%:*} nc=65536
      [[ $val == *:* ]] && nc=${val#*:}
      CORDA_AMD_PARITY_N=$ne CORDA_AMD_PARITY_EC_N=$nc timeout -k 10 1000 python -u -m pytest \
        tests/test_gpu_parity_mix.py -x -v -s --timeout 900 --timeout-method thread > "$O/parity.log" 2>&1 ;;
    ab)
      local an=${val%%@*} aa= tag=${val//[:@ ]/_}
      [[ $val == *@* ]] && aa=$(args_of "${val#*@}")
      AB_NAMES="$(args_of "$an")" AB_ARGS="$aa" bash -c 'rm -f gpurun_out/ab.txt && bash tools/ab_bench.sh $AB_NAMES' \
        > "$O/ab_$tag.log" 2>&1 && cp gpurun_out/ab.txt "$O/ab_$tag.txt" ;;
    *)
      echo "unknown step $step" >&2; return 2 ;;
  esac
  local rc=$?
  echo "== $step rc=$rc ($(date +%T))"
  return $rc
}

for s in "$@"; do
  run_step "$s" || exit $?
done
