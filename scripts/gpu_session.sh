#!/bin/bash
# One GPU session: parity tests, then engine probes (C2 variants, C5).
# Every GPU step has its own time limit; the first failure ends the session.
#   TESTS="tests/x.py ..."  test selection (default: every -m gpu test)
#   SKIP_TESTS / SKIP_C2 / SKIP_C5, RUN_BENCH=1 BENCH_ARGS="..."
#   C5_VARIANTS="MILP_DEVICE_SOLVE=off ..." (probe.py --variants)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
echo "start $(date +%T)"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-$R/tests} -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
fi
if [ -z "$SKIP_C2" ]; then
  MILP_PHASE_TIMING=1 timeout -k 10 600 python -u $R/scripts/probe.py --config c2 --steps 20 \
    --variants ${C2_VARIANTS:-"MILP_DENSE_UNROLL=8" "MILP_DENSE_UNROLL=16"} \
    > $OUT/probe_c2.json 2> $OUT/probe_c2.err || { echo "c2 probe failed"; tail -30 $OUT/probe_c2.err; exit 1; }
  cat $OUT/probe_c2.json
fi
if [ -z "$SKIP_C5" ]; then
  MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=${C5_EVERY:-1000} timeout -k 10 600 python -u $R/scripts/probe.py --config c5 --m 100000 --n 1000000 \
    --warmup ${C5_WARMUP:-20000} --steps ${C5_STEPS:-1000} ${C5_VARIANTS:+--variants $C5_VARIANTS} \
    > $OUT/probe_c5.json 2> $OUT/probe_c5.err || { echo "c5 probe failed"; tail -30 $OUT/probe_c5.err; exit 1; }
  cat $OUT/probe_c5.json
fi
if [ -n "$RUN_BENCH" ]; then
  timeout -k 10 900 python -u $R/bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
echo "done $(date +%T)"
