#!/bin/bash
# Round 4: default bench line on the final tree, and the smoke.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_bench2
mkdir -p $OUT
cd $R
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; grep "\[bench" $OUT/bench.err | tail -12
exit $rc
