#!/bin/bash
# End-of-milestone evidence: rocprofv3 summaries (C2, C5, C4), the GPU parity
# suite, then the default bench.py run with the fresh traffic figures.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
if [ -z "$SKIP_PROFILE" ]; then
  TAG=${TAG:-r01_v6} WORKLOADS=${WORKLOADS:-"c2 c5 c4"} bash $R/scripts/gpu_profile.sh > $OUT/profile.log 2>&1 || { echo "profile failed"; tail -30 $OUT/profile.log; exit 1; }
  tail -3 $OUT/profile.log
fi
if [ -n "$SKIP_BENCH" ]; then exit 0; fi
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 900 python -u bench.py --traffic-json ${TRAFFIC_DIR:-$OUT/profiles}/traffic_c2.json --c5-traffic-json ${TRAFFIC_DIR:-$OUT/profiles}/traffic_c5.json > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
