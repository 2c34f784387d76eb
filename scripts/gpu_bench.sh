#!/bin/bash
# Full-size bench (config 2) + rocprofv3 kernel trace + HBM counter passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT/prof
STEPS=${STEPS:-20}
echo "start $(date +%T)"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -m pytest $R/tests -m gpu -x -q > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
fi
timeout -k 10 900 python $R/bench.py --steps $STEPS --warmup 3 > $OUT/bench_full.log 2> $OUT/bench_full.err || { echo "bench failed"; tail -20 $OUT/bench_full.err; exit 1; }
cat $OUT/bench_full.log
echo "bench done $(date +%T)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof/trace -o run -- python3 $R/bench.py --steps $STEPS --warmup 3 --no-cpu > $OUT/prof_trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/prof_trace.log; exit 1; }
echo "trace done $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/prof/fetch -o run -- python3 $R/bench.py --steps $STEPS --warmup 3 --no-cpu > $OUT/prof_fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/prof_fetch.log; exit 1; }
echo "fetch done $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/prof/write -o run -- python3 $R/bench.py --steps $STEPS --warmup 3 --no-cpu > $OUT/prof_write.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/prof_write.log; exit 1; }
echo "all done $(date +%T)"
find $OUT/prof -name "*.csv" | head -20
