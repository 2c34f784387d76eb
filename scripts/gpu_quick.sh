#!/bin/bash
# Parity tests + phase-timed C2 bench (no CPU baseline, no profiling).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -m pytest $R/tests -m gpu -x -q > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
MILP_PHASE_TIMING=1 timeout -k 10 400 python $R/bench.py --steps ${STEPS:-60} --warmup 3 --no-cpu > $OUT/phase.log 2> $OUT/phase.err || { echo "bench failed"; tail -20 $OUT/phase.err; exit 1; }
grep -v "^\[bench" $OUT/phase.err
cat $OUT/phase.log
