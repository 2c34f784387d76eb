#!/bin/bash
# Round 3 final: the whole -m gpu suite and smoke() on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_final
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread \
  2>&1 | tee $OUT/gpu_tests.log | grep -E "passed|failed|error" ; rc=${PIPESTATUS[0]}
echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
exit $rc
