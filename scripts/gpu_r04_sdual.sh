#!/bin/bash
# Round 4: sdual kernel iteration: the device-segment GPU tests (parity with
# the oracle), then a config-4 probe with the device phase profile.
# OUT=<dir under gpurun_out> (default r04_sdual).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${OUT:-r04_sdual}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_sdual_gpu.py tests/test_cpsat.py -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
MILP_SDUAL_PROFILE=1 timeout -k 10 200 python3 -u scripts/probe_batch.py --node --lps 1024 \
  --workers 1024 > $OUT/c4_w1024.json 2> $OUT/c4_w1024.err
rc=$?; echo "probe rc=$rc"; grep -B1 -A40 "sdual profile" $OUT/c4_w1024.err | head -45
exit $rc
