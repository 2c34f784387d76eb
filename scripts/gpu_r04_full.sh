#!/bin/bash
# Round 4: the whole GPU suite on the current tree, then the config-4 probe
# with the device phase profile. OUT=<dir under gpurun_out>.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${OUT:-r04_full}
mkdir -p $OUT
cd $R
timeout -k 10 1500 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests -m gpu > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
MILP_SDUAL_PROFILE=1 timeout -k 10 200 python3 -u scripts/probe_batch.py --node --lps 1024 \
  --workers 1024 > $OUT/c4_w1024.json 2> $OUT/c4_w1024.err
rc=$?; echo "probe rc=$rc"; grep -A12 "sdual profile" $OUT/c4_w1024.err
exit $rc
