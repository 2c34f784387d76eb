#!/bin/bash
# Round 3, last check of the committed tree: the whole GPU suite, smoke() and the
# default bench, each under its own time limit; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_last
mkdir -p $O
timeout -k 10 660 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u $R/bench.py > $O/bench.json 2> $O/bench.log
rc=$?; echo "bench rc=$rc"; exit $rc
