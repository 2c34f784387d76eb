#!/bin/bash
# Config-5 study on one MI355X: phase-timed probe variants, a rocprofv3
# kernel trace of the C5 bench section, then a test selection with durations.
#   VARIANTS="... ..." (probe.py --variants), SKIP_PROF, TESTS="..." (none: skip)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
echo "start $(date +%T)"
MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=1000 timeout -k 10 300 python -u $R/scripts/probe.py --config c5 \
  --m 100000 --n 1000000 --warmup 20000 --steps 1000 --variants ${VARIANTS:-"" "MILP_DEVICE_SOLVE=off"} \
  > $OUT/probe_c5.json 2> $OUT/probe_c5.err || { echo "probe failed"; tail -30 $OUT/probe_c5.err; exit 1; }
cat $OUT/probe_c5.json
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5 -o run -- python3 $R/bench.py --no-c2 --no-c3 --batch-lps 0 --no-cpu \
    > $OUT/prof_c5.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_c5.log; exit 1; }
  tail -1 $OUT/prof_c5.log
fi
if [ -n "$TESTS" ]; then
  cd $R
  MILP_WATCHDOG_S=30 timeout -k 10 ${TEST_LIMIT:-700} python -u -m pytest $TESTS -m gpu -x -v --durations=0 \
    --timeout 240 --timeout-method thread > $OUT/gpu_tests_part.log 2>&1 \
    || { echo "gpu tests failed"; grep -E "FAILED|Error|watchdog|Timeout" $OUT/gpu_tests_part.log | head -20; tail -40 $OUT/gpu_tests_part.log; exit 1; }
  tail -50 $OUT/gpu_tests_part.log
fi
echo "done $(date +%T)"
