# round-end rehearsal on the current tree: whole GPU suite, smoke(), default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:?tag}
O=gpurun_out/final_$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
