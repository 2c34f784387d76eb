#!/bin/bash
# Round 4, first GPU session: the sdual pool after the ring rework (sdual
# GPU tests incl. the bench-scale and wrap-around cases), the CP-SAT batch
# test, a config-4 probe with the finer device phase profile, then the
# default bench with the new C5 windows.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_a
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_sdual_gpu.py tests/test_cpsat.py -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
MILP_SDUAL_PROFILE=1 timeout -k 10 200 python3 -u scripts/probe_batch.py --node --lps 1024 \
  --workers 1024 > $OUT/c4_w1024.json 2> $OUT/c4_w1024.err
rc=$?; echo "probe rc=$rc"; grep -A40 "sdual profile" $OUT/c4_w1024.err | head -45
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.log
rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.log
exit $rc
