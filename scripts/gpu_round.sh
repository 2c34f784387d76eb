#!/bin/bash
# Round check on one MI355X: smoke, bench (N=1 defaults), then the -m gpu
# suite. Every GPU step has its own time limit; the first failure ends it.
#   SKIP_SMOKE / SKIP_BENCH / SKIP_TESTS, TESTS="...", BENCH_ARGS="..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
echo "start $(date +%T)"
if [ -z "$SKIP_SMOKE" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python -u $R/bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
if [ -z "$SKIP_TESTS" ]; then
  MILP_WATCHDOG_S=${WATCHDOG:-30} timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest ${TESTS:-$R/tests} -m gpu -x -v \
    --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { echo "gpu tests failed"; grep -E "FAILED|Error|watchdog" $OUT/gpu_tests.log | head -20; tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
fi
echo "done $(date +%T)"
